#include <stdlib.h>
/* link stubs for the GPU back ends: the ASan harness runs the host code with the CPU oracles only */
void *h265_hip_backend_create(){return 0;} void *m2dec_amd_hip_backend_create(){return 0;} int m2dec_amd_hip_backend_timing(){return 0;}
void *m2v_hip_create(){return 0;} void m2v_hip_destroy(){} int m2v_hip_set_frames(){return 0;} int m2v_hip_submit(){return 0;} int m2v_hip_sync(){return 0;}

/* pinned record arenas of the parse jobs (runtime.hip): plain heap memory here */
void *m2dec_amd_pinned_alloc(size_t n) { return malloc(n); }
void m2dec_amd_pinned_free(void *p) { free(p); }

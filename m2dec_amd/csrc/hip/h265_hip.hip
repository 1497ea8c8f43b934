/* placeholder: replaced by the gfx950 H.265 reconstruction */
#include <hip/hip_runtime.h>
#include "m2d_recon.h"
#include "h265_dec.h"
extern "C" int h265_hip_backend_create(h265r_backend_t *out, int device) { (void)out; (void)device; return -1; }
extern "C" int m2dec_amd_h265_hip_backend_create(h265r_backend_t *out, int device) { return h265_hip_backend_create(out, device); }

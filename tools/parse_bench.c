/* Host parse throughput of the H.264 path alone (null back end: no reconstruction), with hardware
 * counters where the kernel exposes them: tools/parse_bench.c <stream.264> [reps] */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <sys/ioctl.h>
#include <sys/syscall.h>
#include <linux/perf_event.h>
#include "m2dec_amd.h"
static int pe(unsigned type, unsigned long long cfg){struct perf_event_attr a;memset(&a,0,sizeof a);a.type=type;a.size=sizeof a;a.config=cfg;a.disabled=1;a.exclude_kernel=1;a.exclude_hv=1;return (int)syscall(__NR_perf_event_open,&a,0,-1,-1,0);}
int main(int argc,char**argv){
  FILE*f=fopen(argv[1],"rb"); fseek(f,0,SEEK_END); long n=ftell(f); fseek(f,0,SEEK_SET); unsigned char*d=malloc(n); if(fread(d,1,n,f)!=(size_t)n) return 1; fclose(f);
  int reps=argc>2?atoi(argv[2]):3;
  int fi=pe(PERF_TYPE_HARDWARE,PERF_COUNT_HW_INSTRUCTIONS), fc=pe(PERF_TYPE_HARDWARE,PERF_COUNT_HW_CPU_CYCLES), fb=pe(PERF_TYPE_HARDWARE,PERF_COUNT_HW_BRANCH_MISSES);
  if(fi<0){perror("perf_event_open");}
  for(int r=0;r<reps;r++){ m2r_backend_t be; m2dec_amd_null_backend_create(&be);
    if(fi>=0){ioctl(fi,PERF_EVENT_IOC_RESET,0);ioctl(fc,PERF_EVENT_IOC_RESET,0);ioctl(fb,PERF_EVENT_IOC_RESET,0);ioctl(fi,PERF_EVENT_IOC_ENABLE,0);ioctl(fc,PERF_EVENT_IOC_ENABLE,0);ioctl(fb,PERF_EVENT_IOC_ENABLE,0);}
    struct timespec t0,t1; clock_gettime(CLOCK_MONOTONIC,&t0);
    int fr=m2dec_amd_decode_stream3(d,n,&be,0,-1,0,NULL,NULL,NULL);
    clock_gettime(CLOCK_MONOTONIC,&t1);
    long long ins=0,cyc=0,bm=0; if(fi>=0){ioctl(fi,PERF_EVENT_IOC_DISABLE,0);ioctl(fc,PERF_EVENT_IOC_DISABLE,0);ioctl(fb,PERF_EVENT_IOC_DISABLE,0);if(read(fi,&ins,8)<0||read(fc,&cyc,8)<0||read(fb,&bm,8)<0)return 1;}
    be.destroy(be.self);
    printf("%.3f ms/frame  %d frames  Minstr/frame %.2f  Mcyc/frame %.2f  Kbrmiss/frame %.1f\n",((t1.tv_sec-t0.tv_sec)*1e3+(t1.tv_nsec-t0.tv_nsec)/1e6)/fr,fr,ins/1e6/fr,cyc/1e6/fr,bm/1e3/fr);}
  return 0;}

// Output-write microbenchmark on tmpfs (/dev/shm): N MiB written by T threads with pwrite (mode 0),
// or copied into a MAP_SHARED mapping (1), populated first (2), fallocated first (3).
//   gcc -O2 -pthread -o w tools/tmpfs_write.c && ./w 1024 8 0
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <unistd.h>
#include <pthread.h>
#include <sys/mman.h>
#include <time.h>
static double now(){struct timespec t;clock_gettime(CLOCK_MONOTONIC,&t);return t.tv_sec+1e-9*t.tv_nsec;}
static size_t N; static char* src; static int fd; static char* dst; static int T;
static void* pw(void* a){size_t i=(size_t)a, e=N/T; size_t off=i*e; size_t n=e; while(n){ssize_t w=pwrite(fd,src+off,n,off); off+=w;n-=w;} return 0;}
static void* mc(void* a){size_t i=(size_t)a, e=N/T; memcpy(dst+i*e,src+i*e,e); return 0;}
int main(int argc,char**argv){N=(size_t)atol(argv[1])<<20; T=atoi(argv[2]); int mode=atoi(argv[3]);
 src=malloc(N); memset(src,1,N);
 const char* p="/dev/shm/wt_out.bin"; unlink(p);
 double t0=now(); fd=open(p,O_RDWR|O_CREAT|O_TRUNC,0644); pthread_t th[64];
 if(mode==0){ for(int i=0;i<T;i++) pthread_create(&th[i],0,pw,(void*)(size_t)i); for(int i=0;i<T;i++) pthread_join(th[i],0);}
 else { if(ftruncate(fd,N)) return 1; if(mode==3) fallocate(fd,0,0,N); dst=mmap(0,N,PROT_READ|PROT_WRITE,MAP_SHARED|(mode==2?MAP_POPULATE:0),fd,0);
   double t1=now(); for(int i=0;i<T;i++) pthread_create(&th[i],0,mc,(void*)(size_t)i); for(int i=0;i<T;i++) pthread_join(th[i],0); munmap(dst,N); fprintf(stderr,"  (map+populate %.3f)\n", t1-t0);}
 close(fd); double t=now()-t0; printf("mode %d threads %d: %.3f s %.2f GB/s\n",mode,T,t,N/t/1e9); unlink(p); return 0;}

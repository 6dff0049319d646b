// Debug: run observe() on the device for a fixed layout and print the obs.
#include <cstdio>
#include <hip/hip_runtime.h>
#include "env_device.h"
using namespace mm;
__global__ void k(const uint8_t* Lg, float* o, uint8_t* mk, int* nb, int use_lds) {
  __shared__ uint8_t L[64];
  if (threadIdx.x < 49) L[threadIdx.x] = Lg[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    View v; v.L = use_lds ? L : (uint8_t*)Lg; v.w=7; v.h=7; v.ex=6; v.ey=3; v.kx=6; v.ky=5; v.t=0; v.max_t=1200;
    Agent a0{}, a1{}; a0.tag=2; a1.tag=3; a1.x=0;a1.y=0;a1.dir=2;a1.mem=0xffffffffu;a1.exit_len=-1; a0.tfls=0;
    reset_agent(a0,2,0);
    observe(v,a0,a1,false,[&](int i,float x){o[i]=x;},mk);
    nb[0] = rel_nbrs(v,2,2,0);
    nb[1] = rel_nbrs(v,a0.dir,a0.x,a0.y);
  }
}
int main(){
  int lay[7][7]={{8, 1, 4, 4, 8, 1, 8}, {8, 1, 1, 1, 8, 1, 8}, {8, 1, 8, 1, 8, 1, 8}, {8, 1, 8, 1, 8, 1, 16}, {4, 4, 8, 1, 4, 4, 0}, {0, 1, 8, 1, 1, 1, 0}, {0, 1, 4, 4, 4, 4, 0}};
  uint8_t Lh[49]; for(int y=0;y<7;y++)for(int x=0;x<7;x++)Lh[y*7+x]=lay[y][x];
  uint8_t *Ld, *mkd; float* od; int* nbd;
  hipMalloc(&Ld,64); hipMalloc(&od,65*4); hipMalloc(&mkd,8); hipMalloc(&nbd,8);
  hipMemcpy(Ld,Lh,49,hipMemcpyHostToDevice);
  for (int lds=0; lds<2; lds++) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, Ld, od, mkd, nbd, lds);
    float o[65]; uint8_t mk[6]; int nb[2];
    hipMemcpy(o,od,260,hipMemcpyDeviceToHost); hipMemcpy(mk,mkd,6,hipMemcpyDeviceToHost); hipMemcpy(nb,nbd,8,hipMemcpyDeviceToHost);
    printf("lds=%d obs:", lds); for(int i=0;i<12;i++) printf(" %g",o[i]); printf(" mask:"); for(int i=0;i<6;i++) printf(" %d",mk[i]); printf(" nb %d %d\n", nb[0], nb[1]);
  }
}

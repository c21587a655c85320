// Which instructions SQ_INSTS_SALU counts on gfx950: one wave per kernel,
// 100 iterations of 16 copies of one instruction (k_base: none).
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP16(x) x x x x x x x x x x x x x x x x
__global__ void k_base(int* o) { int a = o[0]; for (int i = 0; i < 100; ++i) { asm volatile("" : "+v"(a)); } o[1] = a; }
__global__ void k_nop(int* o) { int a = o[0]; for (int i = 0; i < 100; ++i) { asm volatile(REP16("s_nop 0\n") : "+v"(a)); } o[1] = a; }
__global__ void k_wait(int* o) { int a = o[0]; for (int i = 0; i < 100; ++i) { asm volatile(REP16("s_waitcnt lgkmcnt(0)\n") : "+v"(a)); } o[1] = a; }
__global__ void k_sadd(int* o) { int a = o[0]; int s = __builtin_amdgcn_readfirstlane(a); for (int i = 0; i < 100; ++i) { asm volatile(REP16("s_add_u32 %0, %0, 1\n") : "+s"(s)); } o[1] = a + s; }
__global__ void k_rdl(int* o) { int a = o[threadIdx.x]; int s = 0; for (int i = 0; i < 100; ++i) { asm volatile(REP16("v_readlane_b32 %0, %1, 5\n") : "=s"(s) : "v"(a)); a += s; } o[1] = a; }
__global__ void k_exec(int* o) { int a = o[0]; for (int i = 0; i < 100; ++i) { asm volatile(REP16("s_mov_b64 exec, exec\n") : "+v"(a)); } o[1] = a; }
__global__ void k_cbr(int* o) { int a = o[0]; for (int i = 0; i < 100; ++i) { asm volatile(REP16("s_cbranch_execz 0\n") : "+v"(a)); } o[1] = a; }
int main() {
  int* d; hipMalloc(&d, 1024); hipMemset(d, 0, 1024);
  hipLaunchKernelGGL(k_base, dim3(1), dim3(64), 0, 0, d);
  hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, 0, d);
  hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, 0, d);
  hipLaunchKernelGGL(k_sadd, dim3(1), dim3(64), 0, 0, d);
  hipLaunchKernelGGL(k_rdl, dim3(1), dim3(64), 0, 0, d);
  hipLaunchKernelGGL(k_exec, dim3(1), dim3(64), 0, 0, d);
  hipLaunchKernelGGL(k_cbr, dim3(1), dim3(64), 0, 0, d);
  hipDeviceSynchronize();
  printf("probe done\n");
  return 0;
}

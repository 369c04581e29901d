// VALU issue-cost probe (measurement aid, not product code): cycles per wave64 instruction per SIMD
// for the instruction mixes of the filter leaves, at 6 waves per SIMD on every CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)

// K0: 96 independent-ish v_add_u32 per iteration (baseline)
__global__ __launch_bounds__(256) void k_add(uint32_t *out, int iters) {
  uint32_t a = threadIdx.x, b = blockIdx.x, c = 0;
  for (int i = 0; i < iters; i++) {
    asm volatile(REP32("v_add_u32 %0, %0, %1\n\tv_add_u32 %1, %1, %2\n\tv_add_u32 %2, %2, %0\n\t") : "+v"(a), "+v"(b), "+v"(c));
  }
  out[blockIdx.x * 256 + threadIdx.x] = a + b + c;
}
// K1: the filter leaf step: v_sub, v_cmp -> vcc, v_addc (r = 2r + vcc)
__global__ __launch_bounds__(256) void k_leaf(uint32_t *out, int iters) {
  uint32_t w = threadIdx.x * 0x9e3779b9u, r = 0, d;
  const uint32_t lo = 0x30000000u, sp = 0x40000000u;
  for (int i = 0; i < iters; i++) {
    asm volatile(REP32("v_sub_u32 %1, %2, %3\n\tv_cmp_gt_u32 vcc, %4, %1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc\n\t")
                 : "+v"(r), "=&v"(d) : "v"(w), "s"(lo), "s"(sp) : "vcc");
    w += r;
  }
  out[blockIdx.x * 256 + threadIdx.x] = r;
}
// K2: the same compare into 32 separate SGPR-pair masks, no per-lane accumulate
__global__ __launch_bounds__(256) void k_leaf_sgpr(uint32_t *out, int iters) {
  uint32_t w = threadIdx.x * 0x9e3779b9u, d;
  const uint32_t lo = 0x30000000u, sp = 0x40000000u;
  uint64_t acc = 0;
  for (int i = 0; i < iters; i++) {
    uint64_t m;
    asm volatile(REP32("v_sub_u32 %1, %2, %3\n\tv_cmp_gt_u32 %0, %4, %1\n\t")
                 : "=&s"(m), "=&v"(d) : "v"(w), "s"(lo), "s"(sp));
    acc ^= m;
    w += (uint32_t)acc;
  }
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)acc;
}
// K3: alignbit + lshl (window extraction per doc)
__global__ __launch_bounds__(256) void k_align(uint32_t *out, int iters) {
  uint32_t x = threadIdx.x, y = blockIdx.x, f = 0;
  for (int i = 0; i < iters; i++) {
    asm volatile(REP32("v_alignbit_b32 %0, %1, %2, 7\n\tv_lshlrev_b32 %1, 4, %0\n\t") : "+v"(f), "+v"(x), "+v"(y));
  }
  out[blockIdx.x * 256 + threadIdx.x] = f;
}
// K4: v_bfe_u32 + v_med3 + v_cmp_eq -> vcc + addc (alternative formulation)
__global__ __launch_bounds__(256) void k_bfe(uint32_t *out, int iters) {
  uint32_t w = threadIdx.x * 0x9e3779b9u, r = 0, x, m;
  for (int i = 0; i < iters; i++) {
    asm volatile(REP32("v_bfe_u32 %1, %3, 4, 4\n\tv_med3_u32 %2, %1, 3, 9\n\tv_cmp_eq_u32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc\n\t")
                 : "+v"(r), "=&v"(x), "=&v"(m) : "v"(w) : "vcc");
    w += r;
  }
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

typedef void (*kfn)(uint32_t *, int);
int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount, bpc = 6, iters = 2000;
  const int blocks = cus * bpc;
  uint32_t *out;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  struct { const char *name; kfn f; int instrs; } ks[] = {
      {"add x96", k_add, 96}, {"sub+cmp(vcc)+addc x32", k_leaf, 96}, {"sub+cmp(sgpr) x32", k_leaf_sgpr, 64},
      {"alignbit+lshl x32", k_align, 64}, {"bfe+med3+cmp+addc x32", k_bfe, 128}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto &k : ks) {
    k.f<<<blocks, 256>>>(out, iters);
    hipEventRecord(e0);
    k.f<<<blocks, 256>>>(out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // wave-instructions per SIMD = blocks*4 waves / (cus*4 SIMDs) * iters * instrs
    const double per_simd = (double)blocks * 4 / (cus * 4) * iters * k.instrs;
    printf("%-26s %8.3f ms  %.2f ns per wave-instr per SIMD (%.2f cycles @2.4GHz)\n", k.name, ms, ms * 1e6 / per_simd,
           ms * 1e6 / per_simd * 2.4);
  }
  return 0;
}

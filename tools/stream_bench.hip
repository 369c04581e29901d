// Read-streaming ceiling on this GPU for the filter's access shapes (measurement tool, not product code).
//   A  plain global_load_dwordx4, grid-stride, XOR-accumulated (default cache policy)
//   B  same with non-temporal loads
//   C  LDS-DMA (global_load_lds_dwordx4) of `chunk` bytes per step per wave from a contiguous per-wave range,
//      `nbuf` ring slots (nbuf-1 in flight), `wpc` waves per CU -- the filter kernel's staging shape
//   D  the same ring, each step gathering `ncols` column slices of `cb` bytes from `ncols` separate regions (the
//      filter's tile: every scan column's 256 x bits bytes, the last 1 KiB instruction partly masked)
// usage: stream_bench [GiB=1]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void read_plain(const u32x4 *__restrict__ p, size_t n, uint32_t *out, int nt) {
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    u32x4 v = nt ? __builtin_nontemporal_load(p + i) : p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__device__ __forceinline__ void dma16(const void *g, uint32_t lds) {
  __builtin_amdgcn_global_load_lds((const void *)g, (__attribute__((address_space(3))) void *)(uintptr_t)lds, 16, 0, 0);
}

#define VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
__device__ __forceinline__ void wait_vm(int n) {
  switch (__builtin_amdgcn_readfirstlane(n)) {
    VMW(0) VMW(1) VMW(2) VMW(3) VMW(4) VMW(5) VMW(6) VMW(7) VMW(8) VMW(9) VMW(10) VMW(11) VMW(12) VMW(13) VMW(14)
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
}

template <int NBUF>
__global__ __launch_bounds__(256) void read_dma(const uint8_t *__restrict__ p, size_t bytes, int chunk, uint32_t *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * 4, gw = (int64_t)blockIdx.x * 4 + wave;
  const int64_t nch = bytes / chunk;
  const int64_t b = nch * gw / waves, e = nch * (gw + 1) / waves;
  unsigned char *ring = smem + (size_t)wave * NBUF * chunk;
  const uint32_t rl = (uint32_t)(uintptr_t)ring;
  const int per = chunk / 1024;
  int64_t pf = b;
  for (int i = 0; i < NBUF - 1 && pf < e; i++, pf++)
    for (int k = 0; k < per; k++) dma16(p + pf * chunk + k * 1024 + lane * 16, rl + (uint32_t)(((pf - b) % NBUF) * chunk + k * 1024));
  uint32_t acc = 0;
  for (int64_t t = b; t < e; t++) {
    if (pf < e) {
      for (int k = 0; k < per; k++) dma16(p + pf * chunk + k * 1024 + lane * 16, rl + (uint32_t)(((pf - b) % NBUF) * chunk + k * 1024));
      pf++;
      // wait until tile t has landed: (NBUF-1) tiles x per instructions were issued after it
      wait_vm(per * (NBUF - 1));
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    acc ^= ((volatile uint32_t *)(ring + ((t - b) % NBUF) * chunk))[lane];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int NBUF>
__global__ __launch_bounds__(256) void read_dma_cols(const uint8_t *__restrict__ p, size_t bytes, int ncols, int cb,
                                                     uint32_t *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * 4, gw = (int64_t)blockIdx.x * 4 + wave;
  const size_t region = bytes / ncols;
  const int64_t ntiles = region / cb;
  const int64_t b = ntiles * gw / waves, e = ntiles * (gw + 1) / waves;
  const int slot = ((ncols * cb + 1023) / 1024) * 1024;  // ring slot bytes
  unsigned char *ring = smem + (size_t)wave * NBUF * slot;
  const uint32_t rl = (uint32_t)(uintptr_t)ring;
  const int per = (cb + 1023) / 1024;  // instructions per column
  auto issue = [&](int64_t t) {
    const uint32_t dst = rl + (uint32_t)(((t - b) % NBUF) * slot);
    for (int c = 0; c < ncols; c++)
      for (int k = 0; k < per; k++)
        if (k * 1024 + lane * 16 < cb)
          dma16(p + c * region + t * cb + k * 1024 + lane * 16, dst + (uint32_t)(c * cb + k * 1024));  // (uniform base: lane i lands at +16 i)
  };
  int64_t pf = b;
  for (int i = 0; i < NBUF - 1 && pf < e; i++, pf++) issue(pf);
  uint32_t acc = 0;
  for (int64_t t = b; t < e; t++) {
    if (pf < e) {
      issue(pf);
      pf++;
      wait_vm(ncols * per * (NBUF - 1));
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    acc ^= ((volatile uint32_t *)(ring + ((t - b) % NBUF) * slot))[lane];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char **argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 1.0;
  const size_t bytes = (size_t)(gib * (1 << 30)) & ~(size_t)0xffff;
  uint8_t *p;
  uint32_t *out;
  CHECK(hipMalloc(&p, bytes));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(p, 1, bytes));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto time = [&](auto launch, const char *name) {
    for (int w = 0; w < 3; w++) launch();
    CHECK(hipEventRecord(a));
    const int reps = 10;
    for (int r = 0; r < reps; r++) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("%-44s %8.1f GB/s  (%.3f ms)\n", name, bytes / (ms / reps * 1e-3) / 1e9, ms / reps);
  };
  for (int bpc : {4, 8, 16}) {
    char nm[64];
    snprintf(nm, sizeof nm, "plain  blocks/CU=%d", bpc);
    time([&] { read_plain<<<cus * bpc, 256>>>((const u32x4 *)p, bytes / 16, out, 0); }, nm);
    snprintf(nm, sizeof nm, "nt     blocks/CU=%d", bpc);
    time([&] { read_plain<<<cus * bpc, 256>>>((const u32x4 *)p, bytes / 16, out, 1); }, nm);
  }
  struct Cfg { int chunk, bpc, nbuf; };
  const Cfg cfgs[] = {{6144, 3, 2}, {4096, 3, 3}, {2048, 3, 6}, {8192, 2, 2}, {4096, 4, 2}, {4096, 2, 4},
                      {16384, 1, 2}, {8192, 1, 4}, {2048, 6, 3}, {1024, 8, 4}};
  for (const Cfg &c : cfgs) {
    const size_t lds = (size_t)4 * c.nbuf * c.chunk;
    if (lds > 160 * 1024 / c.bpc) continue;
    char nm[96];
    snprintf(nm, sizeof nm, "dma    chunk=%5d waves/CU=%2d nbuf=%d (%3zu KB)", c.chunk, 4 * c.bpc, c.nbuf, lds * c.bpc / 1024);
    auto go = [&] {
      switch (c.nbuf) {
        case 2: read_dma<2><<<cus * c.bpc, 256, lds>>>(p, bytes, c.chunk, out); break;
        case 3: read_dma<3><<<cus * c.bpc, 256, lds>>>(p, bytes, c.chunk, out); break;
        case 4: read_dma<4><<<cus * c.bpc, 256, lds>>>(p, bytes, c.chunk, out); break;
        default: read_dma<6><<<cus * c.bpc, 256, lds>>>(p, bytes, c.chunk, out); break;
      }
    };
    if (lds > 65536) {
      CHECK(hipFuncSetAttribute((const void *)read_dma<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      CHECK(hipFuncSetAttribute((const void *)read_dma<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      CHECK(hipFuncSetAttribute((const void *)read_dma<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      CHECK(hipFuncSetAttribute((const void *)read_dma<6>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    }
    time(go, nm);
  }
  // the filter's multi-column tiles (D): column slice bytes x columns, ring slots, waves per CU
  struct ColCfg { int ncols, cb, bpc, nbuf; };
  const ColCfg ccfgs[] = {{3, 1536, 4, 2}, {3, 1536, 3, 2}, {3, 1536, 2, 4}, {3, 1536, 1, 8}, {3, 768, 4, 4},
                          {4, 1024, 4, 2}, {1, 4096, 4, 2}, {1, 4096, 2, 4}, {3, 2048, 2, 3}, {6, 768, 2, 4},
                          {2, 2048, 4, 2}, {3, 512, 4, 6}};
  for (const ColCfg &c : ccfgs) {
    const int slot = ((c.ncols * c.cb + 1023) / 1024) * 1024;
    const size_t lds = (size_t)4 * c.nbuf * slot;
    if (lds * c.bpc > 160 * 1024) continue;
    char nm[96];
    snprintf(nm, sizeof nm, "cols   %dx%5d B waves/CU=%2d nbuf=%d (%3zu KB)", c.ncols, c.cb, 4 * c.bpc, c.nbuf, lds * c.bpc / 1024);
    auto go = [&] {
      switch (c.nbuf) {
        case 2: read_dma_cols<2><<<cus * c.bpc, 256, lds>>>(p, bytes, c.ncols, c.cb, out); break;
        case 3: read_dma_cols<3><<<cus * c.bpc, 256, lds>>>(p, bytes, c.ncols, c.cb, out); break;
        case 4: read_dma_cols<4><<<cus * c.bpc, 256, lds>>>(p, bytes, c.ncols, c.cb, out); break;
        case 6: read_dma_cols<6><<<cus * c.bpc, 256, lds>>>(p, bytes, c.ncols, c.cb, out); break;
        default: read_dma_cols<8><<<cus * c.bpc, 256, lds>>>(p, bytes, c.ncols, c.cb, out); break;
      }
    };
    for (auto f : {(const void *)read_dma_cols<2>, (const void *)read_dma_cols<3>, (const void *)read_dma_cols<4>,
                   (const void *)read_dma_cols<6>, (const void *)read_dma_cols<8>})
      CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    time(go, nm);
  }
  CHECK(hipFree(p));
  return 0;
}

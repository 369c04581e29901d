// Multi-column LDS-DMA streaming ceiling (measurement tool, not product code): the filter kernel's staging shape
// with its real per-tile column sizes. A wave owns a contiguous tile range; per step it DMAs `group` consecutive
// tiles of each of k columns (column c: `size_c` bytes per tile, its own region, as the forward indexes lie in HBM)
// into a ring of nbuf slots, nbuf-1 steps in flight.
//   usage: stream_bench2 [GiB=1.2]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

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

struct Cols {
  const uint8_t *base[4];
  int size[4];  // bytes per tile
  int k;
};

__global__ __launch_bounds__(256) void read_multi(Cols c, int64_t ntiles, int group, int nbuf, int slot_bytes, uint32_t *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * 4, gw = (int64_t)blockIdx.x * 4 + wave;
  const int64_t nsteps = ntiles / group;
  const int64_t b = nsteps * gw / waves, e = nsteps * (gw + 1) / waves;
  unsigned char *ring = smem + (size_t)wave * nbuf * slot_bytes;
  const uint32_t rl = (uint32_t)(uintptr_t)ring;
  int per = 0;  // DMA instructions per step
  for (int j = 0; j < c.k; j++) per += (c.size[j] * group + 1023) / 1024;
  auto issue = [&](int64_t s) {
    uint32_t off = (uint32_t)(((s - b) % nbuf) * slot_bytes);
    for (int j = 0; j < c.k; j++) {
      const int nb = c.size[j] * group;
      const uint8_t *g = c.base[j] + s * nb;
      for (int o = 0; o < nb; o += 1024)
        if (o + lane * 16 < nb) dma16(g + o + lane * 16, rl + off + (uint32_t)o);
      off += (uint32_t)nb;
    }
  };
  int64_t pf = b;
  for (int i = 0; i < nbuf - 1 && pf < e; i++, pf++) issue(pf);
  uint32_t acc = 0;
  for (int64_t t = b; t < e; t++) {
    if (pf < e) {
      issue(pf);
      pf++;
      wait_vm(per * (nbuf - 1));
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    acc ^= ((volatile uint32_t *)(ring + ((t - b) % nbuf) * slot_bytes))[lane];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char **argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 1.2;
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *out;
  CHECK(hipMalloc(&out, 64));
  hipEvent_t a, bev;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&bev));
  CHECK(hipFuncSetAttribute((const void *)read_multi, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  struct Shape { const char *name; std::vector<int> sizes; };
  const Shape shapes[] = {{"Q1.1 3/4/6-bit", {768, 1024, 1536}}, {"Q1.3 6/3/4/6-bit", {1536, 768, 1024, 1536}},
                          {"one 13-bit column", {3328}}};
  for (const Shape &sh : shapes) {
    int per_tile = 0;
    for (int s : sh.sizes) per_tile += s;
    const int64_t ntiles = (int64_t)(gib * (1 << 30)) / per_tile / 64 * 64;
    Cols c{};
    c.k = (int)sh.sizes.size();
    for (int j = 0; j < c.k; j++) {
      uint8_t *p;
      CHECK(hipMalloc(&p, (size_t)ntiles * sh.sizes[j] + 4096));
      CHECK(hipMemset(p, 1, (size_t)ntiles * sh.sizes[j]));
      c.base[j] = p;
      c.size[j] = sh.sizes[j];
    }
    const double bytes = (double)ntiles * per_tile;
    for (int group : {1, 2, 4}) {
      for (int wpc : {8, 12, 16, 24}) {
        for (int nbuf : {2, 3, 4, 6}) {
          const int slot = per_tile * group;
          const size_t lds = (size_t)4 * nbuf * slot;
          const int bpc = wpc / 4;
          if (lds * bpc > 160 * 1024 || lds > 160 * 1024) continue;
          auto go = [&] { read_multi<<<cus * bpc, 256, lds>>>(c, ntiles, group, nbuf, slot, out); };
          for (int w = 0; w < 3; w++) go();
          CHECK(hipEventRecord(a));
          const int reps = 10;
          for (int r = 0; r < reps; r++) go();
          CHECK(hipEventRecord(bev));
          CHECK(hipEventSynchronize(bev));
          float ms = 0;
          CHECK(hipEventElapsedTime(&ms, a, bev));
          printf("%-18s group=%d waves/CU=%2d nbuf=%d slot=%6d  %7.1f GB/s\n", sh.name, group, wpc, nbuf, slot,
                 bytes / (ms / reps * 1e-3) / 1e9);
        }
      }
    }
    for (int j = 0; j < c.k; j++) CHECK(hipFree((void *)c.base[j]));
  }
  return 0;
}

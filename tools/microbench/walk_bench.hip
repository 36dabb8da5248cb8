// Microbenchmark for the per-tile chain walk of the frame scan (K1 fs_walk):
// isolates staging, the dependent LDS hop loop and the list write-out on a
// synthetic GET_DATA reply stream (192-byte frames) so their costs can be
// read separately.  Build: hipcc --offload-arch=gfx950 -O3 walk_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int S = 16384;
constexpr int TPB = 4;

__host__ __device__ inline uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }

template <int MODE>
__global__ __launch_bounds__(256) void walk(const uint8_t* __restrict__ buf, int64_t n,
                                           int64_t tiles, const int32_t* __restrict__ ent,
                                           uint16_t* __restrict__ list,
                                           int64_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * TPB + wv;
  if (t >= tiles) return;
  uint8_t* sb = smem + wv * (S + 16);
  const int64_t ts = t * S;
  if (MODE != 3) {
    uint4 v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j)
      __builtin_memcpy(&v[j], buf + ts + 16 * (int64_t)(lane + j * 64), 16);
#pragma unroll
    for (int j = 0; j < 16; ++j) *(uint4*)(sb + 16 * (lane + j * 64)) = v[j];
    if (lane == 0) *(uint4*)(sb + S) = make_uint4(0, 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  int32_t cnt = 0;
  if (MODE == 1) {               // lane-0 divergent walk
    if (lane == 0) {
      int32_t c = ent[t];
      while (c < S) {
        const int32_t a = c & ~3;
        const uint32_t lo = *(const uint32_t*)(sb + a);
        const uint32_t hi = *(const uint32_t*)(sb + a + 4);
        const int32_t len = (int32_t)bswap(__builtin_amdgcn_alignbyte(hi, lo, c & 3));
        if (len < 0 || len > 16000000) break;
        ((uint16_t*)sb)[cnt++] = (uint16_t)c;
        c = c + 4 + len;
      }
    }
    cnt = __shfl(cnt, 0, 64);
  } else if (MODE == 2) {        // wave-uniform scalar walk
    int32_t c = __builtin_amdgcn_readfirstlane(ent[t]);
    while (c < S) {
      const int32_t a = c & ~3;
      const uint32_t lo = *(const uint32_t*)(sb + a);
      const uint32_t hi = *(const uint32_t*)(sb + a + 4);
      const int32_t len = __builtin_amdgcn_readfirstlane(
          (int32_t)bswap(__builtin_amdgcn_alignbyte(hi, lo, c & 3)));
      if (len < 0 || len > 16000000) break;
      if (lane == 0) ((uint16_t*)sb)[cnt] = (uint16_t)c;
      ++cnt;
      c = c + 4 + len;
    }
  } else if (MODE == 3) {        // walk straight from global memory
    int32_t c = __builtin_amdgcn_readfirstlane(ent[t]);
    while (c < S) {
      uint32_t w; __builtin_memcpy(&w, buf + ts + c, 4);
      const int32_t len = __builtin_amdgcn_readfirstlane((int32_t)bswap(w));
      if (len < 0 || len > 16000000) break;
      ++cnt;
      c = c + 4 + len;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  if (MODE == 1 || MODE == 2) {
    uint16_t* L = list + t * (S / 4);
    for (int k = lane; k < cnt; k += 64) L[k] = ((uint16_t*)sb)[k];
  }
  if (lane == 0) counts[t] = cnt;
}

int main(int argc, char** argv) {
  const int frame = argc > 1 ? atoi(argv[1]) : 192;
  const int64_t nframes = argc > 2 ? atoll(argv[2]) : (1 << 20);
  const int64_t n = nframes * frame;
  const int64_t tiles = (n + S - 1) / S;
  std::vector<uint8_t> h(n + 64);
  srand(1);
  for (auto& b : h) b = rand() & 0xff;
  for (int64_t i = 0; i < nframes; ++i) {
    const uint32_t be = bswap(frame - 4);
    memcpy(&h[i * frame], &be, 4);
  }
  std::vector<int32_t> ent(tiles);
  for (int64_t t = 0; t < tiles; ++t) {
    const int64_t ts = t * S;
    const int64_t first = (ts + frame - 1) / frame * frame;
    ent[t] = (int32_t)(first - ts);
  }
  uint8_t* d; int32_t* de; uint16_t* dl; int64_t* dc;
  CK(hipMalloc(&d, n + 64)); CK(hipMalloc(&de, tiles * 4));
  CK(hipMalloc(&dl, tiles * (S / 4) * 2)); CK(hipMalloc(&dc, tiles * 8));
  CK(hipMemcpy(d, h.data(), n + 64, hipMemcpyHostToDevice));
  CK(hipMemcpy(de, ent.data(), tiles * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const unsigned grid = (unsigned)((tiles + TPB - 1) / TPB);
  const size_t lds = TPB * (S + 16);
  auto run = [&](auto kern, const char* name, size_t lds_bytes) {
    for (int i = 0; i < 3; ++i) kern<<<grid, 256, lds_bytes>>>(d, n, tiles, de, dl, dc);
    CK(hipEventRecord(a));
    const int R = 10;
    for (int i = 0; i < R; ++i) kern<<<grid, 256, lds_bytes>>>(d, n, tiles, de, dl, dc);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    int64_t c0; CK(hipMemcpy(&c0, dc, 8, hipMemcpyDeviceToHost));
    printf("%-28s %8.1f us  (tile0 frames %lld)\n", name, ms * 1000 / R, (long long)c0);
  };
  printf("frame %d B, %lld frames, %lld tiles\n", frame, (long long)nframes, (long long)tiles);
  run(walk<0>, "stage only", lds);
  run(walk<1>, "stage + lane0 walk", lds);
  run(walk<2>, "stage + uniform walk", lds);
  run(walk<3>, "uniform walk from global", lds);
  run(walk<3>, "global walk, no LDS", 0);
  return 0;
}

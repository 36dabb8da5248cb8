// Phase profile of the frame-scan frontier kernel (fs_frontier) on
// synthetic request (42 B frames) and reply (192 B frames) streams: per-tile
// wall-clock of staging, block-wide rounds, the wave phase and merge
// resolution, plus round / wave-iteration counts.
// Build: hipcc --offload-arch=gfx950 -O3 -DZKMI_FE_PROFILE -I../../csrc/kernels
//        frontier_bench.hip -o frontier_bench
#include "../../csrc/kernels/frame_scan.hip"
#include "../../csrc/kernels/scan.hip"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static void fill(std::vector<uint8_t>& h, int kind, int64_t nframes) {
  srand(7);
  h.clear();
  for (int64_t i = 0; i < nframes; ++i) {
    uint8_t f[256];
    int len;
    if (kind == 0) {                 // GET_DATA request, 25-byte path
      char path[32];
      snprintf(path, sizeof path, "/bench/d%06lld/n%09lld", (long long)(i / 1000),
               (long long)i);
      const int pl = (int)strlen(path);
      len = 4 + 4 + 4 + 4 + pl + 1;
      auto be = [&](int o, uint32_t v) {
        f[o] = v >> 24; f[o + 1] = v >> 16; f[o + 2] = v >> 8; f[o + 3] = v;
      };
      be(0, len - 4); be(4, (uint32_t)i); be(8, 4); be(12, pl);
      memcpy(f + 16, path, pl); f[16 + pl] = 0;
    } else {                         // GET_DATA reply: 100 B data + Stat
      len = 192;
      for (int k = 0; k < len; ++k) f[k] = rand() & 0xff;
      auto be = [&](int o, uint32_t v) {
        f[o] = v >> 24; f[o + 1] = v >> 16; f[o + 2] = v >> 8; f[o + 3] = v;
      };
      be(0, 188); be(4, (uint32_t)i); be(8, 0); be(12, 5000000 + (uint32_t)i); be(16, 0);
      be(20, 100);
      memset(f + 124, 0, 68);        // Stat: mostly zeros / small values
      be(124 + 4, (uint32_t)i + 1); be(124 + 12, (uint32_t)i + 1);
      be(124 + 52, 100);
    }
    h.insert(h.end(), f, f + len);
  }
}

int main(int argc, char** argv) {
  const int64_t nframes = argc > 1 ? atoll(argv[1]) : (1 << 20);
  for (int kind = 0; kind < 2; ++kind) {
    std::vector<uint8_t> h;
    fill(h, kind, nframes);
    const int64_t n = (int64_t)h.size();
    const int64_t tiles = (n + zk::FS_S - 1) / zk::FS_S;
    uint8_t* d; uint16_t* f0; int32_t* surv; uint64_t* prof;
    CK(hipMalloc(&d, n + 64)); CK(hipMalloc(&f0, tiles * zk::FS_W * 2));
    CK(hipMalloc(&surv, tiles * 8)); CK(hipMalloc(&prof, tiles * 64));
    CK(hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice));
    CK(hipMemset(prof, 0, tiles * 64));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(zk::g_fe_prof), &prof, sizeof(prof)));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    constexpr int W = (int)zk::FS_W;
    const size_t lds = zk::fe_lds(W);
    for (int i = 0; i < 2; ++i)
      zk::fs_frontier<W><<<(unsigned)tiles, zk::FE_T, lds>>>(
          d, n, 16 << 20, f0, surv);
    CK(hipEventRecord(a));
    zk::fs_frontier<W><<<(unsigned)tiles, zk::FE_T, lds>>>(
        d, n, 16 << 20, f0, surv);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint64_t> p(tiles * 8);
    CK(hipMemcpy(p.data(), prof, tiles * 64, hipMemcpyDeviceToHost));
    double ph[4] = {0, 0, 0, 0}, rounds = 0, iters = 0, mx_it = 0;
    for (int64_t t = 0; t < tiles; ++t) {
      const uint64_t* q = &p[t * 8];
      for (int k = 0; k < 4; ++k) ph[k] += (double)(q[k + 1] - q[k]);
      rounds += q[5]; iters += q[6]; mx_it = std::max(mx_it, (double)q[6]);
    }
    // wall_clock64 runs at 100 MHz on gfx9: 10 ns per tick
    printf("%s: %lld tiles, kernel %.1f us; per tile avg: stage %.2f us, rounds %.2f us"
           " (%.1f rounds), wave %.2f us (%.1f iters, max %.0f), resolve %.2f us\n",
           kind ? "reply 192B" : "request 42B", (long long)tiles, ms * 1000,
           ph[0] / tiles * 0.01, ph[1] / tiles * 0.01, rounds / tiles,
           ph[2] / tiles * 0.01, iters / tiles, mx_it, ph[3] / tiles * 0.01);
    // survivor walks on the frontier's hand-offs
    uint16_t* list; int32_t* rc;
    CK(hipMalloc(&list, tiles * zk::FE_NSURV * zk::FS_LMAX * 2));
    CK(hipMalloc(&rc, tiles * zk::FE_NSURV * 4));
    for (int v = 0; v < 2; ++v) {
      for (int i = 0; i < 3; ++i) {
        if (i == 2) CK(hipEventRecord(a));
        if (v == 0)
          zk::fs_survivor<<<(unsigned)tiles, 64, zk::FV_LDS>>>(d, n, 16 << 20,
                                                              (int)zk::FS_W, f0,
                                                              surv, list, rc);
        else
          zk::fs_survivor_g<<<(unsigned)((tiles + 3) / 4), 256, 0>>>(
              d, n, 16 << 20, (int)zk::FS_W, tiles, f0, surv, list, rc);
      }
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      std::vector<int32_t> hr(tiles * zk::FE_NSURV);
      CK(hipMemcpy(hr.data(), rc, hr.size() * 4, hipMemcpyDeviceToHost));
      double mean = 0; for (auto x : hr) mean += x; mean /= tiles;
      printf("  %s: %.1f us (avg %.1f frames recorded per tile)\n",
             v ? "fs_survivor_g" : "fs_survivor (LDS)", ms * 1000, mean);
    }
    CK(hipFree(list)); CK(hipFree(rc));
    CK(hipFree(d)); CK(hipFree(f0)); CK(hipFree(surv)); CK(hipFree(prof));
  }
  return 0;
}

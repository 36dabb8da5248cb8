// The MFMA byte-plane prefix sum, as a workgroup-level device function: the
// "MFMA-packed byte scan" of the north star (BASELINE.json), shared by the
// device-wide scan engine (scan.hip scan_apply_mfma) and the one-workgroup
// scans on the GET step's critical path (scan.hip scan_one_block_mfma for
// K10's block sums, tree.hip tree_finish_scan_k for K13's).
//
// A wave owns 1024 values as 16 segments x 64.  Each value is split into
// byte planes; one i8 MFMA (v_mfma_i32_16x16x64_i8) per (plane, quarter)
// multiplies a strictly-lower-triangular ones matrix by 16 segments' bytes,
// giving the in-segment exclusive prefix of 16 positions x 16 segments; the
// planes are recombined with shifts.  Bytes are fed as (b - 128) because
// the operand is signed; the bias is added back per position.  Only the
// planes some value of the wave needs are multiplied (values < 64 KiB: 2
// planes, 8 MFMAs per 1024 values).  A wave holding any value outside
// [0, 2^32) takes a lane-serial path.  Reference hot loop this replaces:
// lib/jute-buffer.js:181-189 (writeLengthPrefixed, one record at a time).
#pragma once
#include "zk_common.h"

namespace zk {

constexpr int MS_V = 16;                        // values per lane
constexpr int MS_WAVE_E = 64 * MS_V;            // 1024 per wave
typedef int v4i __attribute__((ext_vector_type(4)));

// Strictly lower-triangular ones, as this lane's A fragment for quarter q:
// A[i][k] = (k < 16q + i), lane l holding row i = l & 15 and the 16 k's
// 16 (l >> 4) + e.  B uses the same (lane, e) -> k map, so the sum over k is
// exact whatever order the hardware walks the k's in.
ZK_DEV v4i tri_frag(int q, int lane) {
  const int i = lane & 15, k0 = 16 * (lane >> 4), lim = 16 * q + i;
  v4i a;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    uint32_t x = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
      x |= (uint32_t)(k0 + 4 * w + b < lim ? 1 : 0) << (8 * b);
    a[w] = (int)x;
  }
  return a;
}

// LDS staging: 64-value segments padded by 16 bytes, so the 16 lanes of a
// group reading their 16-value runs (ds_read_b128) hit distinct banks.
template <typename T>
ZK_DEV int lds_idx(int x) { return x + (x >> 6) * (int)(16 / sizeof(T)); }

// int64 slots of the LDS staging area for NT threads
template <int NT>
constexpr int ms_stage_slots() {
  return NT * MS_V + (NT * MS_V / 64) * 2;
}

// One chunk of NT * 16 values: in[0, m) (m <= NT * 16) -> out[0, m) =
// base + exclusive prefix; returns the chunk's sum (every thread).  `stage`
// (ms_stage_slots<NT>() int64) and `wsum` (NT / 64 + 1) are LDS.  Every
// thread of the workgroup calls it.
template <typename T, int NT>
ZK_DEV int64_t mfma_scan_chunk(const T* __restrict__ in, int64_t m,
                               int64_t* __restrict__ out, int64_t base_in,
                               int64_t* stage, int64_t* wsum) {
  constexpr int64_t MS_E = (int64_t)NT * MS_V;
  T* const tin = reinterpret_cast<T*>(stage);
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int j = lane & 15, g = lane >> 4;        // segment, lane group
  const bool full = m >= MS_E;

  // 1. coalesced global -> LDS
#pragma unroll
  for (int k = 0; k < MS_V; ++k) {
    const int x = tid + k * NT;
    tin[lds_idx<T>(x)] = (full || x < m) ? in[x] : (T)0;
  }
  __syncthreads();

  // 2. my 16-value run: segment j of wave w, values 16 g .. 16 g + 15
  const int r0 = w * 1024 + 64 * j + 16 * g;
  int64_t v[MS_V];
  int64_t s = 0;
  uint64_t orv = 0;
#pragma unroll
  for (int e = 0; e < MS_V; ++e) {
    v[e] = (int64_t)tin[lds_idx<T>(r0 + e)];
    s += v[e];
    orv |= (uint64_t)v[e];
  }

  // segment prefix over the 4 lane groups, then over the 16 segments
  const int64_t s0 = __shfl(s, j, 64), s1 = __shfl(s, j + 16, 64),
                s2 = __shfl(s, j + 32, 64), s3 = __shfl(s, j + 48, 64);
  const int64_t seg_tot = s0 + s1 + s2 + s3;
  const int64_t pre_g = (g > 0 ? s0 : 0) + (g > 1 ? s1 : 0) + (g > 2 ? s2 : 0);
  const int64_t seg_inc = wave_incl_scan(lane < 16 ? seg_tot : 0);
  const int64_t seg_base = __shfl(seg_inc, j, 64) - seg_tot;
  const int64_t wave_tot = __shfl(seg_inc, 15, 64);
  uint64_t wor = orv;                            // wave-uniform OR
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) wor |= __shfl_xor(wor, d, 64);

  // wave totals -> block prefix (this barrier also frees `stage`)
  if (lane == 0) wsum[w] = wave_tot;
  __syncthreads();
  int64_t wpre = base_in, ctot = 0;
  for (int x = 0; x < NT / 64; ++x) {
    if (x < w) wpre += wsum[x];
    ctot += wsum[x];
  }
  const int64_t base = wpre + seg_base;          // segment j's start
  const int sbase = w * 1024 + 64 * j;           // segment j in `stage`

  // 3. prefixes -> LDS (int64 slots)
  if (wor >> 32) {
    // some value needs > 32 bits (or is negative): lane-serial, in the
    // layout this lane loaded
    int64_t p = base + pre_g;
#pragma unroll
    for (int e = 0; e < MS_V; ++e) {
      stage[lds_idx<int64_t>(r0 + e)] = p;
      p += v[e];
    }
  } else {
    const int planes = (wor >> 24) ? 4 : (wor >> 16) ? 3 : (wor >> 8) ? 2 : 1;
    // B fragments: plane p of my 16 values, biased to signed bytes
    v4i bfr[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint32_t byte = (uint32_t)(v[4 * w4 + b] >> (8 * p)) & 255u;
          x |= ((byte - 128u) & 255u) << (8 * b);
        }
        bfr[p][w4] = (int)x;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const v4i a = tri_frag(q, lane);
      int64_t acc[4] = {0, 0, 0, 0};
      for (int p = 0; p < planes; ++p) {
        const v4i z = {0, 0, 0, 0};
        const v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bfr[p], z, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int pos = 16 * q + 4 * g + r;    // row of D = position
          acc[r] += (int64_t)(d[r] + 128 * pos) << (8 * p);
        }
      }
      // D layout (16x16): col = lane & 15 (segment j), row = 4 (lane >> 4) + r
#pragma unroll
      for (int r = 0; r < 4; ++r)
        stage[lds_idx<int64_t>(sbase + 16 * q + 4 * g + r)] = base + acc[r];
    }
  }
  __syncthreads();

  // 4. coalesced LDS -> global
#pragma unroll
  for (int k = 0; k < MS_V; ++k) {
    const int x = tid + k * NT;
    if (full || x < m) out[x] = stage[lds_idx<int64_t>(x)];
  }
  __syncthreads();                               // stage / wsum reusable
  return ctot;
}

// One workgroup scans any n: chunks of NT * 16 values with a running
// carry.  Returns the total (every thread).
template <typename T, int NT>
ZK_DEV int64_t mfma_scan_block(const T* __restrict__ in, int64_t n,
                               int64_t* __restrict__ out, int64_t* stage,
                               int64_t* wsum) {
  constexpr int64_t E = (int64_t)NT * MS_V;
  int64_t carry = 0;
  for (int64_t c0 = 0; c0 < n; c0 += E)          // (uniform)
    carry += mfma_scan_chunk<T, NT>(in + c0, min(n - c0, E), out + c0, carry,
                                    stage, wsum);
  return carry;
}

// mfma_scan_chunk without the LDS staging: each lane loads its 16-value run
// straight from global memory (128 contiguous bytes of int64) and stores
// its 16 prefixes back the same way; only the wave totals go through LDS
// (`wsum`, NT / 64 + 1).  For the one-workgroup scans of a few thousand
// values, where the 17-33 KiB staging area made the workgroup wait for a
// CU with that much LDS free beside the other connection's kernels.
template <int NT>
ZK_DEV int64_t mfma_scan_chunk_direct(const int64_t* __restrict__ in,
                                      int64_t m, int64_t* __restrict__ out,
                                      int64_t base_in, int64_t* wsum) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int r0 = w * 1024 + 64 * j + 16 * g;
  int64_t v[MS_V];
  int64_t s = 0;
  uint64_t orv = 0;
  if (r0 + MS_V <= m) {
    const int4* q = reinterpret_cast<const int4*>(in + r0);
#pragma unroll
    for (int e = 0; e < MS_V / 2; ++e) {
      const int4 x = q[e];
      v[2 * e] = (int64_t)((uint64_t)(uint32_t)x.x | (uint64_t)(uint32_t)x.y << 32);
      v[2 * e + 1] =
          (int64_t)((uint64_t)(uint32_t)x.z | (uint64_t)(uint32_t)x.w << 32);
    }
  } else {
#pragma unroll
    for (int e = 0; e < MS_V; ++e) v[e] = r0 + e < m ? in[r0 + e] : 0;
  }
#pragma unroll
  for (int e = 0; e < MS_V; ++e) {
    s += v[e];
    orv |= (uint64_t)v[e];
  }
  const int64_t s0 = __shfl(s, j, 64), s1 = __shfl(s, j + 16, 64),
                s2 = __shfl(s, j + 32, 64), s3 = __shfl(s, j + 48, 64);
  const int64_t seg_tot = s0 + s1 + s2 + s3;
  const int64_t pre_g = (g > 0 ? s0 : 0) + (g > 1 ? s1 : 0) + (g > 2 ? s2 : 0);
  const int64_t seg_inc = wave_incl_scan(lane < 16 ? seg_tot : 0);
  const int64_t seg_base = __shfl(seg_inc, j, 64) - seg_tot;
  const int64_t wave_tot = __shfl(seg_inc, 15, 64);
  uint64_t wor = orv;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) wor |= __shfl_xor(wor, d, 64);
  if (lane == 0) wsum[w] = wave_tot;
  __syncthreads();
  int64_t wpre = base_in, ctot = 0;
  for (int x = 0; x < NT / 64; ++x) {
    if (x < w) wpre += wsum[x];
    ctot += wsum[x];
  }
  __syncthreads();                               // wsum reusable
  const int64_t base = wpre + seg_base;
  int64_t p[MS_V];
  if (wor >> 32) {
    int64_t a = base + pre_g;
#pragma unroll
    for (int e = 0; e < MS_V; ++e) {
      p[e] = a;
      a += v[e];
    }
  } else {
    // the MFMA gives position 16 q + 4 g + r of segment j to this lane; the
    // lane owns positions 16 g .. 16 g + 15 of the same segment: the
    // 4 x 4 results move between the segment's four lanes by shuffles
    const int planes = (wor >> 24) ? 4 : (wor >> 16) ? 3 : (wor >> 8) ? 2 : 1;
    v4i bfr[4];
#pragma unroll
    for (int pl = 0; pl < 4; ++pl) {
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint32_t byte = (uint32_t)(v[4 * w4 + b] >> (8 * pl)) & 255u;
          x |= ((byte - 128u) & 255u) << (8 * b);
        }
        bfr[pl][w4] = (int)x;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const v4i a = tri_frag(q, lane);
      int64_t acc[4] = {0, 0, 0, 0};
      for (int pl = 0; pl < planes; ++pl) {
        const v4i z = {0, 0, 0, 0};
        const v4i dd =
            __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bfr[pl], z, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int pos = 16 * q + 4 * g + r;
          acc[r] += (int64_t)(dd[r] + 128 * pos) << (8 * pl);
        }
      }
      // positions 16 q + 4 g' + r sit in lane j + 16 g'; this lane (group g)
      // owns positions 16 g + 4 k + r, i.e. quarter q == g, from lane
      // j + 16 k: gather them when q == g
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t x = __shfl(acc[r], j + 16 * kk, 64);
          if (q == g) p[4 * kk + r] = base + x;
        }
      }
    }
  }
  if (r0 + MS_V <= m) {
    int4* o = reinterpret_cast<int4*>(out + r0);
#pragma unroll
    for (int e = 0; e < MS_V / 2; ++e)
      o[e] = int4{(int)(uint32_t)p[2 * e], (int)((uint64_t)p[2 * e] >> 32),
                  (int)(uint32_t)p[2 * e + 1],
                  (int)((uint64_t)p[2 * e + 1] >> 32)};
  } else {
#pragma unroll
    for (int e = 0; e < MS_V; ++e)
      if (r0 + e < m) out[r0 + e] = p[e];
  }
  return ctot;
}

template <int NT>
ZK_DEV int64_t mfma_scan_block_direct(const int64_t* __restrict__ in,
                                      int64_t n, int64_t* __restrict__ out,
                                      int64_t* wsum) {
  constexpr int64_t E = (int64_t)NT * MS_V;
  int64_t carry = 0;
  for (int64_t c0 = 0; c0 < n; c0 += E)          // (uniform)
    carry += mfma_scan_chunk_direct<NT>(in + c0, min(n - c0, E), out + c0,
                                        carry, wsum);
  return carry;
}

}  // namespace zk

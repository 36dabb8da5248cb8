// K1 — parallel length-prefixed frame scan.
//
// Reference: ZKDecodeStream._transform (lib/zk-streams.js:39-65) walks the
// i32-BE length chain one frame at a time and memmoves the remainder per
// packet (O(bytes x packets)).  The chain is inherently
// sequential; we make it parallel without speculation errors, in three
// launches over 16 KiB tiles:
//
//  A  fs_frontier  one block per tile: a merging frontier walk from the W
//                  window entry points (the only places a chain can enter
//                  a tile when frames are <= W bytes) -> per-entry exit code
//                  table f0 and ONE surviving walker (all others ended or
//                  merged into it).
//  B  fs_survivor_r  one wave per tile walks the survivor to the tile end
//                  through a 4 KiB LDS ring, records its frame starts, and
//                  summarises the tile: its exit is "constant" when every
//                  non-terminal entry leaves at one position.
//  C  fs_chain     one wave per tile, tiles in order (atomic counter),
//                  decoupled look-back: the constant exit of the tile
//                  before is this tile's entry (validated through the
//                  look-back, repaired when a frame longer than the window
//                  breaks it), a short walk joins the survivor's path, the
//                  inclusive frame count comes from a 64-tile-wide look-back,
//                  and the tile writes its (body offset, length) rows.
//
// The stream length is read on the device (zk_frame_scan3's n_dev, e.g. an
// encoder's total), the grids cover the buffer capacity and tiles past the
// length return at once.  BAD_LENGTH is reported at the exact frame
// (result[1] = its offset, result[2] = 1), the consumed prefix ends at the
// last complete frame, and a partial trailing frame is left for the next
// call (carry), like the reference's buffer.  The round-1 composition path
// (fs_compose / fs_top / fs_down / fs_join + a count scan, 13-15 launches)
// stays selectable for A/B runs (ZKMI_FS_SCAN=compose, host lengths).
#include "zk_common.h"

extern "C" int zk_scan_excl_i64(const int64_t*, int64_t*, int64_t, int64_t*,
                                int64_t*, hipStream_t);
extern "C" int64_t zk_scan_workspace(int64_t);

namespace zk {

constexpr int64_t FS_S = 16384;          // tile bytes
constexpr int64_t FS_W = 2048;           // window (entry points) per tile
constexpr int FS_G = 16;                 // fan-in per composition level
constexpr int FS_MAXL = 6;               // levels (16 KiB * 16^5 = 16 GiB)
constexpr int FS_TOPMAX = 16;            // serial walk bound at the top
constexpr int FS_T = 1024;               // threads per tile workgroup
constexpr int64_t TERM = (int64_t)1 << 62;
constexpr int64_t NONE = -1;
constexpr uint16_t F0_TERM = 0x8000;     // | rel position (< 16384)
constexpr uint16_t F0_ESC = 0xFFFF;      // exit beyond next tile: walk

struct FsCtx {
  const uint8_t* buf;
  int64_t n;
  int64_t maxp;
  int64_t W;                       // window: entry points per unit (<= FS_W)
  int levels;                      // number of levels (>= 1)
  int64_t usize[FS_MAXL];          // unit size in bytes per level
  int64_t units[FS_MAXL];          // unit count per level
  const uint16_t* f0;              // [units0][W]
  int64_t* fl[FS_MAXL];            // [units_l][W] for l >= 1 (absolute)
  int64_t* ent[FS_MAXL];           // entry position per unit (or NONE)
};

// LATE: composition stopped at position pos (a landing outside the next
// unit's window, i.e. after a frame > W bytes).  Only the walkers that follow
// the TRUE chain (fs_top / fs_down) resolve it, by walking on from pos; the
// composition of the ~2000 speculative entry points per unit never walks
// bytes, so a garbage chain that merges into the real one outside a window
// costs one table lookup instead of a hop-by-hop global-memory walk.
constexpr int64_t LATE = (int64_t)1 << 61;

ZK_DEV bool is_term(int64_t v) { return (v & TERM) != 0; }
ZK_DEV bool is_late(int64_t v) { return (v & LATE) != 0; }
ZK_DEV int64_t pos_of(int64_t v) { return v & ~(TERM | LATE); }

// The scanned length: a producer's device-side byte count clamped to the
// buffer capacity (null: the capacity itself, a host-known length).
ZK_DEV int64_t stream_len(const int64_t* n_dev, int64_t n_cap) {
  if (n_dev == nullptr) return n_cap;
  const int64_t v = *n_dev;
  return v < 0 ? 0 : (v < n_cap ? v : n_cap);
}

// One step of the chain in global memory.
ZK_DEV int64_t next_global(const FsCtx& c, int64_t P) {
  if (P >= c.n) return TERM | c.n;
  if (P + 4 > c.n) return TERM | P;
  const int32_t len = ld_be32(c.buf + P);
  if (len < 0 || (int64_t)len > c.maxp) return TERM | P;
  const int64_t nx = P + 4 + len;
  if (nx > c.n) return TERM | P;
  return nx >= c.n ? (TERM | c.n) : nx;
}

ZK_DEV int64_t walk_until(const FsCtx& c, int64_t P, int64_t end) {
  while (!is_term(P) && P < end) P = next_global(c, P);
  return P;
}

// Apply unit u of level L to position P (inside u).  RES = resolve: walk
// bytes / LATE values to the exact result (true-chain walkers); !RES =
// stop with LATE at the first position no table covers (composition).
template <int L, bool RES>
ZK_DEV int64_t apply_unit(const FsCtx& c, int64_t u, int64_t P) {
  if (is_term(P) || is_late(P)) return P;
  if (P >= c.n) return TERM | c.n;
  const int64_t us = u * c.usize[L];
  const int64_t ue = min(us + c.usize[L], c.n);
  const int64_t off = P - us;
  if constexpr (L == 0) {
    if (off < c.W) {
      const uint16_t v = c.f0[u * c.W + off];
      if (v == F0_ESC) return RES ? walk_until(c, P, ue) : (LATE | P);
      if (v & F0_TERM) return TERM | (us + (v & 0x7FFF));
      const int64_t x = us + FS_S + v;
      return x >= c.n ? (TERM | c.n) : x;
    }
    return RES ? walk_until(c, P, ue) : (LATE | P);
  } else {
    if (off < c.W) {
      const int64_t v = c.fl[L][u * c.W + off];
      if (!RES || !is_late(v)) return v;
      P = pos_of(v);                      // resume the true chain here
    } else if (!RES) {
      return LATE | P;
    }
    while (!is_term(P) && P < ue) {
      const int64_t sub = P / c.usize[L - 1];
      P = apply_unit<L - 1, RES>(c, sub, P);
    }
    return P;
  }
}

template <bool RES>
ZK_DEV int64_t apply_level(const FsCtx& c, int l, int64_t u, int64_t P) {
  switch (l) {
    case 0: return apply_unit<0, RES>(c, u, P);
    case 1: return apply_unit<1, RES>(c, u, P);
    case 2: return apply_unit<2, RES>(c, u, P);
    case 3: return apply_unit<3, RES>(c, u, P);
    case 4: return apply_unit<4, RES>(c, u, P);
    default: return apply_unit<5, RES>(c, u, P);
  }
}

// Stage tile bytes [ts, ts+S+16) into LDS (zero beyond n) with NT threads
// (thread index `tid`).  Full tiles issue ALL their 16-byte loads before the
// first LDS write: a load -> wait -> ds_write loop serialises one HBM
// latency per iteration (it made staging the dominant cost of the walks).
template <int NT>
ZK_DEV void stage_tile(const uint8_t* buf, int64_t n, int64_t ts, uint8_t* sb,
                       int tid) {
  constexpr int CH = (int)(FS_S / 16);        // + one pad chunk at CH
  constexpr int PER = CH / NT;
  static_assert(CH % NT == 0, "tile chunks must split evenly");
  if (ts + FS_S + 16 <= n) {
    uint4 v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j)
      __builtin_memcpy(&v[j], buf + ts + 16 * (int64_t)(tid + j * NT), 16);
    uint4 pad = make_uint4(0, 0, 0, 0);
    if (tid == 0) __builtin_memcpy(&pad, buf + ts + FS_S, 16);
#pragma unroll
    for (int j = 0; j < PER; ++j) *(uint4*)(sb + 16 * (tid + j * NT)) = v[j];
    if (tid == 0) *(uint4*)(sb + FS_S) = pad;
    return;
  }
  const int64_t lim = min(FS_S + 4, n - ts);
  for (int k = tid; k < FS_S + 16; k += NT)
    sb[k] = k < lim ? buf[ts + k] : 0;
}

// A' (default) — the same f0 table by a MERGING FRONTIER WALK instead of
// pointer jumping over all 16 Ki positions.  One walker per window entry
// e < W starts at e; every round each live walker takes one hop in the
// staged tile and claims the position it lands on in an owner table.  A
// walker that lands on a claimed position has the same future as the
// claimant: it stops and records "merged into <claimant>".  Walkers end on
// a terminal (bad length / partial frame) or on leaving the tile.
// Afterwards merge links are resolved by pointer jumping over W entries.
//
// Work is O(W + positions claimed) instead of O(S log S): in real streams
// nearly every speculative entry dies or leaves the tile on its first hop
// (ASCII or random bytes read as a length are huge) and the rest merge into
// the true chain within a few hops, so after 1-3 block-wide rounds <= 64
// walkers remain and wave 0 finishes them alone, one LDS round trip per hop
// (owner word and next length read together), no block barriers.  The walk
// is bounded: each hop claims a fresh position, so <= S hops in total.
constexpr int FE_T = 256;
// LDS of fs_frontier<W>: staged tile, owner table, W results, hand-off area
// Windows of <= 256 entries keep walker ids in bytes plus a claimed-bit
// map ("narrow" owner table: 18 KiB instead of 32 KiB, and only the 2 KiB
// bit map is zeroed per tile), so a CU holds 4 frontier blocks, not 3.
constexpr bool fe_narrow(int W) { return W <= 256; }
inline size_t fe_lds(int W) {
  const size_t own = fe_narrow(W) ? FS_S + FS_S / 8 : FS_S * 2;
  return (FS_S + 16) + own + (size_t)W * 2 + 66 * 4;
}

// Owner table of fs_frontier: get(q) = claiming walker id + 1, 0 = none.
// Narrow: set() writes the id byte, then ORs the claimed bit with release
// order; get() reads the bit with acquire order, then the byte, so a bit
// seen set always comes with its (last) writer's byte.  Wide: one uint16
// per position, written and read whole.
template <bool NARROW>
struct FeOwners {
  uint8_t* base;                     // NARROW: [S] bytes, then [S/32] bits
  ZK_DEV uint32_t* bits() const { return (uint32_t*)(base + FS_S); }
  ZK_DEV uint32_t get(int32_t q) const {
    if constexpr (NARROW) {
      const uint32_t w = __hip_atomic_load(&bits()[q >> 5], __ATOMIC_ACQUIRE,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
      if (!((w >> (q & 31)) & 1u)) return 0;
      return (uint32_t)*(volatile const uint8_t*)(base + q) + 1u;
    } else {
      return ((const uint16_t*)base)[q];
    }
  }
  // re-read by the lane that just claimed q (its own bit is set)
  ZK_DEV uint32_t get_claimed(int32_t q) const {
    if constexpr (NARROW)
      return (uint32_t)*(volatile const uint8_t*)(base + q) + 1u;
    else
      return *(volatile const uint16_t*)((const uint16_t*)base + q);
  }
  ZK_DEV void set(int32_t q, int32_t e) const {
    if constexpr (NARROW) {
      *(volatile uint8_t*)(base + q) = (uint8_t)e;
      __hip_atomic_fetch_or(&bits()[q >> 5], 1u << (q & 31),
                            __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      ((uint16_t*)base)[q] = (uint16_t)(e + 1);
    }
  }
  // zero before use (narrow: the bits only)
  ZK_DEV void clear(int tid, int nt) const {
    const int n16 = NARROW ? FS_S / 128 : FS_S / 8;
    uint4* z = NARROW ? (uint4*)bits() : (uint4*)base;
    for (int k = tid; k < n16; k += nt) z[k] = make_uint4(0, 0, 0, 0);
  }
};
constexpr uint16_t F0_MERGE = 0x4000;        // | parent walker id (< 2048)

ZK_DEV bool f0_is_merge(uint16_t v) { return (v & 0xF800) == F0_MERGE; }

// Phase timestamps of fs_frontier for tools/microbench/frontier_bench.hip
// (compiled in only with -DZKMI_FE_PROFILE).
#ifdef ZKMI_FE_PROFILE
__device__ uint64_t* g_fe_prof;
#define FE_MARK(k) do { if (threadIdx.x == 0 && g_fe_prof) \
    g_fe_prof[blockIdx.x * 8 + (k)] = wall_clock64(); } while (0)
#define FE_NOTE(k, v) do { if (threadIdx.x == 0 && g_fe_prof) \
    g_fe_prof[blockIdx.x * 8 + (k)] = (v); } while (0)
#else
#define FE_MARK(k) do {} while (0)
#define FE_NOTE(k, v) do {} while (0)
#endif

// One hop from tile-relative p.  Returns the f0 code when the walk ends
// here (terminal / leaves the tile), else 0xFFFE and q (in-tile successor).
constexpr uint16_t FE_GO = 0xFFFE;
constexpr uint16_t FE_PENDING = 0xFFFD;      // | ... slot s = 0xFFFD - s
#ifndef ZKMI_FE_NSURV
#define ZKMI_FE_NSURV 1
#endif
constexpr int FE_NSURV = ZKMI_FE_NSURV;      // survivors handed off per tile
ZK_DEV uint16_t fe_pending(int slot) { return (uint16_t)(FE_PENDING - slot); }
ZK_DEV uint16_t fe_hop(uint32_t lo, uint32_t hi, int32_t p, int32_t nrel,
                       int32_t maxp, int32_t& q) {
  // 32-bit throughout: p < 2^14, len <= maxp <= 2^30, nrel clamped to 2^30
  const int32_t len = (int32_t)bswap32(__builtin_amdgcn_alignbyte(hi, lo,
                                                                  p & 3));
  const int32_t nx = p + 4 + len;
  if ((p + 4 > nrel) | (len < 0) | (len > maxp) | (nx > nrel))
    return (uint16_t)(F0_TERM | p);
  if (nx >= FS_S) {
    const int32_t x = nx - (int32_t)FS_S;
    return x < 0x4000 ? (uint16_t)x : F0_ESC;
  }
  q = nx;
  return FE_GO;
}

// fe_hop for a length already extracted (wave-uniform walks: the length is
// built in VALU and moved to an SGPR once, instead of moving both words).
ZK_DEV uint16_t fe_hop_len(int32_t len, int32_t p, int32_t nrel, int32_t maxp,
                           int32_t& q) {
  const int32_t nx = p + 4 + len;
  if ((p + 4 > nrel) | (len < 0) | (len > maxp) | (nx > nrel))
    return (uint16_t)(F0_TERM | p);
  if (nx >= FS_S) {
    const int32_t x = nx - (int32_t)FS_S;
    return x < 0x4000 ? (uint16_t)x : F0_ESC;
  }
  q = nx;
  return FE_GO;
}

ZK_DEV int32_t fe_len(uint32_t lo, uint32_t hi, int32_t p) {
  return (int32_t)bswap32(__builtin_amdgcn_alignbyte(hi, lo, p & 3));
}

ZK_DEV void fe_words(const uint8_t* sb, int32_t p, uint32_t& lo, uint32_t& hi) {
  const int32_t a = p & ~3;
  lo = *(const uint32_t*)(sb + a);
  hi = *(const uint32_t*)(sb + a + 4);
}

// One 256-thread block per tile.  Block-wide rounds (8 walkers per thread,
// LDS reads batched) run while more than 64 walkers live; then wave 0 moves
// the survivors one per lane and hops them together, claiming positions,
// until one is left; that one is handed to fs_survivor.  Merge links are
// then resolved (entries rooted at the survivor become FE_PENDING).
// (A wave-per-tile variant without barriers was slower: 53 KiB of LDS per
// tile leaves 3 waves per CU, too few to hide the LDS latency chains.)
//
// The stream length is n = min(*n_dev, n_cap) (n_dev may be null: n_cap):
// the grid covers the capacity and tiles at or past n leave at once, so a
// producer's device-side byte count bounds the scan without a host read and
// no stale byte past it is walked.  When `lbw` is given (one-pass chain,
// fs_chain) every block also zeroes its tile's look-back words and block 0
// the result and the chain's tile counter.
template <int W>
__global__ __launch_bounds__(FE_T) void fs_frontier(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ n_dev,
    int64_t n_cap, int64_t maxp, uint16_t* __restrict__ f0,
    int32_t* __restrict__ surv, uint64_t* __restrict__ lbw,
    int64_t* __restrict__ result) {
  constexpr int FE_K = W / FE_T;             // walkers per thread (1..8)
  static_assert(W % FE_T == 0 && FE_K >= 1 && FE_K <= 8, "window");
  constexpr bool NARROW = fe_narrow(W);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* sb = smem;                                      // [S + 16]
  const FeOwners<NARROW> own{smem + FS_S + 16};            // owner table
  uint16_t* res = (uint16_t*)(smem + FS_S + 16 +
                              (NARROW ? FS_S + FS_S / 8 : FS_S * 2));  // [W]
  uint32_t* hand = (uint32_t*)(res + W);                   // [64] + 2 ctrs
  const int64_t t = blockIdx.x;
  FE_MARK(0);
  const int64_t n = stream_len(n_dev, n_cap);
  if (lbw != nullptr) {
    if (threadIdx.x < 2) lbw[2 * t + threadIdx.x] = 0;
    if (t == 0 && threadIdx.x >= 64 && threadIdx.x < 68)
      result[threadIdx.x - 64] = 0;
    if (t == 0 && threadIdx.x >= 128 && threadIdx.x < 132)
      lbw[2 * (int64_t)gridDim.x + threadIdx.x - 128] = 0;
  }
  const int64_t ts = t * FS_S;
  if (ts >= n) {
    if (threadIdx.x < FE_NSURV) surv[t * FE_NSURV + threadIdx.x] = -1;
    return;
  }
  const int32_t nrel = (int32_t)min(n - ts, (int64_t)1 << 30);
  const int32_t maxp32 = (int32_t)min(maxp, (int64_t)1 << 30);
  stage_tile<FE_T>(buf, n, ts, sb, threadIdx.x);
  own.clear(threadIdx.x, FE_T);
  if (threadIdx.x < 2) hand[64 + threadIdx.x] = 0;
  __syncthreads();
  int32_t pos[FE_K], nq[FE_K];
  uint32_t act = 0;
#pragma unroll
  for (int k = 0; k < FE_K; ++k) {
    const int32_t e = threadIdx.x + k * FE_T;
    pos[k] = e;
    own.set(e, e);
    act |= 1u << k;
  }
  __syncthreads();
  FE_MARK(1);
  // ---- block-wide rounds while many walkers live ------------------------
  int nrounds = 0;
  for (int r = 0;; ++r) {
    ++nrounds;
    // phase 1: hop, then claim the landing position (racy; phase 2 decides).
    // All of a thread's LDS reads are issued before any of its writes, so
    // the 8 walkers' round trips overlap instead of chaining.
    uint32_t lo[FE_K], hi[FE_K];
#pragma unroll
    for (int k = 0; k < FE_K; ++k)
      if (act & (1u << k)) fe_words(sb, pos[k], lo[k], hi[k]);
    uint16_t code[FE_K];
#pragma unroll
    for (int k = 0; k < FE_K; ++k) {
      nq[k] = 0;
      code[k] = (act & (1u << k))
                    ? fe_hop(lo[k], hi[k], pos[k], nrel, maxp32, nq[k])
                    : FE_GO;
    }
    uint32_t o[FE_K];
#pragma unroll
    for (int k = 0; k < FE_K; ++k)
      o[k] = ((act & (1u << k)) && code[k] == FE_GO) ? own.get(nq[k]) : 0;
#pragma unroll
    for (int k = 0; k < FE_K; ++k) {
      if (!(act & (1u << k))) continue;
      const int32_t e = threadIdx.x + k * FE_T;
      if (code[k] != FE_GO) {
        res[e] = code[k];
        act &= ~(1u << k);
      } else if (o[k] != 0) {
        res[e] = (uint16_t)(F0_MERGE | (o[k] - 1));
        act &= ~(1u << k);
      } else {
        own.set(nq[k], e);
      }
    }
    if (__popc(act)) atomicAdd(&hand[64 + (r & 1)], (uint32_t)__popc(act));
    __syncthreads();
    const uint32_t live = hand[64 + (r & 1)];
    if (threadIdx.x == 0) hand[64 + ((r + 1) & 1)] = 0;
    // phase 2: the last writer of own[q] owns it; the others merge into it
    uint32_t o2[FE_K];
#pragma unroll
    for (int k = 0; k < FE_K; ++k) o2[k] = (act & (1u << k)) ? own.get(nq[k]) : 0;
#pragma unroll
    for (int k = 0; k < FE_K; ++k) {
      if (!(act & (1u << k))) continue;
      const int32_t e = threadIdx.x + k * FE_T;
      if (o2[k] != (uint32_t)(e + 1)) {
        res[e] = (uint16_t)(F0_MERGE | (o2[k] - 1));
        act &= ~(1u << k);
      } else {
        pos[k] = nq[k];
      }
    }
    if (live <= 64) break;
    __syncthreads();                    // counter reset visible next round
  }
  FE_MARK(2);
  FE_NOTE(5, nrounds);
  // ---- hand the survivors to wave 0 ---------------------------------------
  __syncthreads();
  if (threadIdx.x == 0) hand[64] = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < FE_K; ++k) {
    if (!(act & (1u << k))) continue;
    const uint32_t slot = atomicAdd(&hand[64], 1u);
    hand[slot] = ((uint32_t)(threadIdx.x + k * FE_T) << 16) | (uint32_t)pos[k];
  }
  __syncthreads();
  if (threadIdx.x < FE_NSURV) surv[t * FE_NSURV + threadIdx.x] = -1;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int cnt = (int)hand[64];
    bool a = lane < cnt;
    int32_t e = 0, p = 0;
    if (a) {
      e = (int32_t)(hand[lane] >> 16);
      p = (int32_t)(hand[lane] & 0xFFFF);
    }
    int iters = 0;
    for (;;) {
      const uint64_t am = __ballot(a);
      if (am == 0) break;
      ++iters;
      FE_NOTE(6, iters);
      if (__popcll(am) <= FE_NSURV) {
        // one or two walkers left (the usual case after a few hops): hand
        // them to fs_survivor, which walks them without the owner table (a
        // second survivor is typically a garbage chain running beside the
        // true one for a long way without merging)
        if (a) {
          const int slot = __builtin_amdgcn_mbcnt_hi(
              (uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0));
          res[e] = fe_pending(slot);
          surv[t * FE_NSURV + slot] = (e << 16) | p;
        }
        break;
      }
      int32_t q = 0;
      bool claim = false;
      uint32_t ow = 0;
      if (a) {
        uint32_t lo, hi;
        fe_words(sb, p, lo, hi);
        const uint16_t code = fe_hop(lo, hi, p, nrel, maxp32, q);
        if (code != FE_GO) {
          res[e] = code;
          a = false;
        } else {
          ow = own.get(q);
          claim = true;
        }
      }
      if (claim && ow != 0) {
        res[e] = (uint16_t)(F0_MERGE | (ow - 1));
        a = false;
        claim = false;
      }
      if (claim) own.set(q, e);
      if (__popcll(__ballot(claim)) > 1) {
        // several lanes may have claimed the same q: LDS ops of a wave
        // execute in order, so this re-read sees every lane's write
        if (claim) {
          // volatile: the compiler must not forward this lane's own store
          const uint32_t o2 = own.get_claimed(q);
          if (o2 != (uint32_t)(e + 1)) {
            res[e] = (uint16_t)(F0_MERGE | (o2 - 1));
            a = false;
            claim = false;
          }
        }
      }
      if (claim) p = q;
    }
  }
  __syncthreads();
  FE_MARK(3);
  // ---- resolve merge links: the links are final now, so no barriers: each
  // thread advances its 8 entries (LDS reads overlapping) and writes every
  // step back, so chains compress for everyone (racy but monotone pointer
  // jumping).  Chains are long: every window start is a walker, so in a
  // stream of 42-byte frames ~48 starts merge one into the next along the
  // true chain; following them hop by hop cost ~17 us per tile.  Entries
  // rooted at a survivor end at fe_pending(slot), which fs_survivor
  // replaces with its final code.
  {
    uint16_t v[FE_K];
#pragma unroll
    for (int k = 0; k < FE_K; ++k) v[k] = res[threadIdx.x + k * FE_T];
    for (;;) {
      bool any = false;
#pragma unroll
      for (int k = 0; k < FE_K; ++k)
        if (f0_is_merge(v[k])) { v[k] = res[v[k] & 0x7FF]; any = true; }
#pragma unroll
      for (int k = 0; k < FE_K; ++k) res[threadIdx.x + k * FE_T] = v[k];
      if (!any) break;
    }
    uint16_t* out = f0 + t * W;
#pragma unroll
    for (int k = 0; k < FE_K; ++k) out[threadIdx.x + k * FE_T] = v[k];
  }
  FE_MARK(4);
}

// Level l -> l+1: fl[l+1][u][p] = position after leaving unit u from us+p.
__global__ __launch_bounds__(FS_T) void fs_compose(FsCtx c, int l) {
  const int64_t u = blockIdx.x;
  const int64_t us = u * c.usize[l + 1];
  const int64_t ue = min(us + c.usize[l + 1], c.n);
  for (int64_t p = threadIdx.x; p < c.W; p += blockDim.x) {
    int64_t P = us + p;
    if (P >= c.n) P = TERM | c.n;
    while (!is_term(P) && P < ue) {
      const int64_t sub = P / c.usize[l];
      P = apply_level<false>(c, l, sub, P);
    }
    c.fl[l + 1][u * c.W + p] = P;
  }
}

// Staged composition / push-down: a parent's FS_G child tables are pulled
// into LDS in one parallel burst, so the dependent chain of child lookups
// runs at LDS latency instead of one global round trip per child (these
// chains were the whole cost of fs_compose / fs_down).  Level-0 rows are the
// uint16 f0 codes, higher levels the int64 fl positions; a level whose rows
// do not fit FS_STAGE_MAX uses the global kernels above.
constexpr size_t FS_STAGE_MAX = 64 * 1024;

inline size_t fs_stage_bytes(int l, int64_t W) {
  return (size_t)FS_G * (size_t)W * (l == 0 ? 2 : 8);
}

template <bool RES>
ZK_DEV int64_t apply_staged(const FsCtx& c, int l, int64_t s, int64_t P,
                            const uint16_t* t16, const int64_t* t64) {
  if (is_term(P) || is_late(P)) return P;
  if (P >= c.n) return TERM | c.n;
  const int64_t us = s * c.usize[l];
  const int64_t off = P - us;
  if (off >= c.W) return RES ? apply_level<true>(c, l, s, P) : (LATE | P);
  if (l == 0) {
    const uint16_t v = t16[off];
    if (v == F0_ESC) return RES ? apply_level<true>(c, 0, s, P) : (LATE | P);
    if (v & F0_TERM) return TERM | (us + (v & 0x7FFF));
    const int64_t x = us + FS_S + v;
    return x >= c.n ? (TERM | c.n) : x;
  }
  const int64_t v = t64[off];
  if (!RES || !is_late(v)) return v;
  return apply_level<true>(c, l, s, P);    // LATE: resolve via global tables
}

// Pull the child rows [s0, s1) of level l into LDS (zero rows past s1).
ZK_DEV void stage_children(const FsCtx& c, int l, int64_t s0, int64_t s1,
                           uint8_t* lds) {
  const int64_t W = c.W;
  const int64_t es = l == 0 ? 2 : 8;
  const int64_t nvec = (s1 - s0) * W * es / 16;
  const uint4* src = l == 0 ? (const uint4*)(c.f0 + s0 * W)
                            : (const uint4*)(c.fl[l] + s0 * W);
  for (int64_t k = threadIdx.x; k < nvec; k += blockDim.x)
    ((uint4*)lds)[k] = src[k];
}

__global__ __launch_bounds__(FS_T) void fs_compose_staged(FsCtx c, int l) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int64_t u = blockIdx.x;
  const int64_t us = u * c.usize[l + 1];
  const int64_t ue = min(us + c.usize[l + 1], c.n);
  const int64_t s0 = u * FS_G;
  const int64_t s1 = min(s0 + FS_G, c.units[l]);
  stage_children(c, l, s0, s1, lds);
  __syncthreads();
  const uint16_t* t16 = (const uint16_t*)lds;
  const int64_t* t64 = (const int64_t*)lds;
  for (int64_t p = threadIdx.x; p < c.W; p += blockDim.x) {
    int64_t P = us + p;
    if (P >= c.n) P = TERM | c.n;
    while (!is_term(P) && P < ue) {
      const int64_t sub = P / c.usize[l];
      const int64_t r = (sub - s0) * c.W;
      P = apply_staged<false>(c, l, sub, P, t16 + r, t64 + r);
    }
    c.fl[l + 1][u * c.W + p] = P;
  }
}

// One wave per parent: stage its children, lane 0 walks them.
__global__ __launch_bounds__(64) void fs_down_staged(FsCtx c, int l) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int64_t u = blockIdx.x;
  const int64_t s0 = u * FS_G;
  const int64_t s1 = min(s0 + FS_G, c.units[l]);
  stage_children(c, l, s0, s1, lds);
  __syncthreads();
  if (threadIdx.x != 0) return;
  const uint16_t* t16 = (const uint16_t*)lds;
  const int64_t* t64 = (const int64_t*)lds;
  int64_t P = c.ent[l + 1][u];
  for (int64_t s = s0; s < s1; ++s) {
    const int64_t ss = s * c.usize[l];
    const int64_t se = min(ss + c.usize[l], c.n);
    if (P != NONE && !is_term(P) && P >= ss && P < se) {
      c.ent[l][s] = P;
      const int64_t r = (s - s0) * c.W;
      P = apply_staged<true>(c, l, s, P, t16 + r, t64 + r);
    } else {
      c.ent[l][s] = NONE;
    }
  }
}

// Serial walk over the top level; writes entries and the final status.
__global__ void fs_top(FsCtx c, int64_t* __restrict__ result) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int L = c.levels - 1;
  int64_t P = c.n > 0 ? 0 : (TERM | 0);
  for (int64_t u = 0; u < c.units[L]; ++u) {
    const int64_t us = u * c.usize[L];
    const int64_t ue = min(us + c.usize[L], c.n);
    if (!is_term(P) && P >= us && P < ue) {
      c.ent[L][u] = P;
      P = apply_level<true>(c, L, u, P);
    } else {
      c.ent[L][u] = NONE;
    }
  }
  const int64_t q = pos_of(P);
  result[1] = q;                       // consumed / stop position
  int64_t bad = 0;
  if (q + 4 <= c.n) {
    const int32_t len = ld_be32(c.buf + q);
    if (len < 0 || (int64_t)len > c.maxp) bad = 1;
  }
  result[2] = bad;
}

// Push entries from level l+1 down to level l (one thread per parent).
__global__ void fs_down(FsCtx c, int l) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= c.units[l + 1]) return;
  int64_t P = c.ent[l + 1][u];
  const int64_t s0 = u * FS_G;
  const int64_t s1 = min(s0 + FS_G, c.units[l]);
  for (int64_t s = s0; s < s1; ++s) {
    const int64_t ss = s * c.usize[l];
    const int64_t se = min(ss + c.usize[l], c.n);
    if (P != NONE && !is_term(P) && P >= ss && P < se) {
      c.ent[l][s] = P;
      P = apply_level<true>(c, l, s, P);
    } else {
      c.ent[l][s] = NONE;
    }
  }
}

constexpr int64_t FS_LMAX = FS_S / 4;    // most frame starts a tile can hold

// ---- frontier pipeline, stages 2-4 -----------------------------------------
// Survivor of tile t: surv[t] = (walker id << 16) | position, or -1; its
// frame starts R go to list[t*FS_LMAX ...], their count to rcount[t].

// Wave-wide min / max of a 32-bit value.
ZK_DEV uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, d, 64));
  return v;
}
ZK_DEV uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d, 64));
  return v;
}

// Replace fe_pending(slot) in the tile's f0 row by the slot's final code and
// summarise the patched row: the tile's exit is CONSTANT when every entry
// whose chain does not end in the tile (terminal codes are ignored: a true
// chain entering there makes the stream bad before any later tile matters)
// leaves it at one position.  Returns that absolute position, or -1 (two
// exits, an ESC code, or every entry terminal).  Every real stream tile has
// a constant exit unless a frame is longer than the window: all the true
// frame starts in the window merge within a hop or two.
ZK_DEV int64_t fe_patch_row(uint16_t* row, int W, int lane,
                            const uint16_t fin[FE_NSURV], int64_t ts) {
  uint32_t lo = 0x10000u, hi = 0u;
  bool esc = false;
  for (int j = lane; j < W / 8; j += 64) {
    uint4 v = ((const uint4*)row)[j];
    uint16_t* h = (uint16_t*)&v;
    bool any = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int sl = 0; sl < FE_NSURV; ++sl)
        if (h[k] == fe_pending(sl)) { h[k] = fin[sl]; any = true; }
      const uint16_t c = h[k];
      if (c == F0_ESC) {
        esc = true;
      } else if (!(c & F0_TERM)) {
        lo = min(lo, (uint32_t)c);
        hi = max(hi, (uint32_t)c + 1u);
      }
    }
    if (any) ((uint4*)row)[j] = v;
  }
  lo = wave_min_u32(lo);
  hi = wave_max_u32(hi);
  if (__ballot(esc) != 0 || lo == 0x10000u || hi != lo + 1u) return -1;
  return ts + FS_S + (int64_t)lo;
}

// A2'' fs_survivor_r (default): the LDS walk of fs_survivor through a 4 KiB
// ring instead of the whole staged tile.  The survivor only moves forward,
// so the ring holds the 2 KiB chunk it walks in and the next one; the chunk
// after that is prefetched into registers (32 bytes per lane) while the
// walk runs and written into the ring slot just vacated when the walk
// crosses a chunk boundary (a frame longer than a chunk restages at its
// landing point).  4 KiB of LDS per tile lets a CU hold as many walks as it
// holds waves (32) instead of the 9 the 16 KiB tile allowed, so every tile
// of a 42 MB request stream walks in one round (2688 tiles, formerly two
// LDS rounds), and the 12288 tiles of a 192 MB reply stream walk with LDS
// hop latency instead of L2 latency.  The hot loop is fs_survivor's, with
// the chunk end folded into its position bound.
constexpr int FR_CH = 2048;                  // ring chunk (bytes)
constexpr int FR_RING = 2 * FR_CH;
constexpr int FR_KMAX = (int)(FS_S / FR_CH);  // last chunk (bytes past tile)

// Chunk k (tile-relative bytes [k*CH, (k+1)*CH)) of the tile at ts: 32 bytes
// per lane, zero past the stream end.
ZK_DEV void fr_load(const uint8_t* __restrict__ buf, int64_t n, int64_t ts,
                    int k, int lane, uint4& a, uint4& b) {
  const int64_t g = ts + (int64_t)k * FR_CH + lane * 32;
  if (g + 32 <= n) {
    __builtin_memcpy(&a, buf + g, 16);
    __builtin_memcpy(&b, buf + g + 16, 16);
    return;
  }
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t x = 0;
    for (int q = 0; q < 4; ++q) {
      const int64_t y = g + 4 * j + q;
      if (y < n) x |= (uint32_t)buf[y] << (8 * q);
    }
    w[j] = x;
  }
  a = make_uint4(w[0], w[1], w[2], w[3]);
  b = make_uint4(w[4], w[5], w[6], w[7]);
}

ZK_DEV void fr_store(uint8_t* ring, int k, int lane, const uint4& a,
                     const uint4& b) {
  uint8_t* d = ring + (k & 1) * FR_CH + lane * 32;
  *(uint4*)d = a;
  *(uint4*)(d + 16) = b;
}

ZK_DEV int32_t fr_len(const uint8_t* ring, int32_t c) {
  const int32_t a = c & ~3;
  const uint32_t lo = *(const uint32_t*)(ring + (a & (FR_RING - 1)));
  const uint32_t hi = *(const uint32_t*)(ring + ((a + 4) & (FR_RING - 1)));
  return __builtin_amdgcn_readfirstlane(fe_len(lo, hi, c));
}

//
// fs_survive is the walk itself (one wave, tile t): it records the
// survivor's frame starts in list[t], their count in rcount[t], patches and
// summarises the tile's f0 row, and returns the speculated exit (the
// survivor's exit when it leaves the tile, else the constant-row exit, -1
// when there is none) and the survivor's end `send`: the absolute position
// its last frame leaves the tile at, or TERM | pos (| TBAD when the length
// at pos is invalid rather than cut off by the stream end), -1 without a
// survivor.  The survivor is the chain nearly every window entry merged
// into; a garbage entry whose random "length" jumps out of the tile makes
// the f0 row non-constant in most real tiles, so the constant-row rule is
// only the fallback for tiles without one.
constexpr int64_t TBAD = (int64_t)1 << 60;

ZK_DEV int64_t fs_survive(const uint8_t* __restrict__ buf, int64_t n,
                          int64_t maxp, int32_t W, uint16_t* __restrict__ f0,
                          const int32_t* __restrict__ surv,
                          uint16_t* __restrict__ list,
                          int32_t* __restrict__ rcount, int64_t t,
                          uint8_t* ring, int lane, int64_t& send) {
  const int64_t ts = t * FS_S;
  // one survivor per tile (FE_NSURV == 1; the launcher checks)
  const int32_t sv = __builtin_amdgcn_readfirstlane(surv[t * FE_NSURV]);
  if (sv < 0) {
    if (lane == 0) rcount[t * FE_NSURV] = 0;
    const uint16_t none[FE_NSURV] = {0};
    send = -1;
    return fe_patch_row(f0 + t * W, W, lane, none, ts);
  }
  const int32_t nrel = (int32_t)min(n - ts, (int64_t)1 << 30);
  const int32_t maxp32 = (int32_t)min(maxp, (int64_t)1 << 30);
  const uint32_t umax = (uint32_t)maxp32;
  const int32_t lim = min(nrel + 1, (int32_t)FS_S);
  uint16_t* L = list + t * FE_NSURV * FS_LMAX;
  int32_t c = sv & 0xFFFF;
  int32_t lo = c / FR_CH;                       // ring = chunks lo, lo + 1
  uint4 pa, pb;                                 // prefetched chunk lo + 2
  {
    uint4 a0, b0, a1, b1;
    fr_load(buf, n, ts, lo, lane, a0, b0);
    fr_load(buf, n, ts, lo + 1, lane, a1, b1);
    fr_store(ring, lo, lane, a0, b0);
    fr_store(ring, lo + 1, lane, a1, b1);
    if (lo + 2 <= FR_KMAX) fr_load(buf, n, ts, lo + 2, lane, pa, pb);
  }
  int32_t m = 0;
  uint32_t ent = 0;
  for (;;) {
    const int32_t bound = min(lim, (lo + 1) * FR_CH);
    for (;;) {                                  // hot: hops inside chunk lo
      const int32_t len = fr_len(ring, c);
      const int32_t nx = c + 4 + len;
      if (((uint32_t)len > umax) | (nx >= bound)) break;
      ent = lane == (m & 63) ? (uint32_t)c : ent;
      ++m;
      if ((m & 63) == 0) L[m - 64 + lane] = (uint16_t)ent;
      c = nx;
    }
    const int32_t len = fr_len(ring, c);
    const int32_t nx = c + 4 + len;
    if (((uint32_t)len > umax) | (nx >= lim)) break;   // the ending hop
    // a clean hop out of chunk lo (still inside the tile)
    ent = lane == (m & 63) ? (uint32_t)c : ent;
    ++m;
    if ((m & 63) == 0) L[m - 64 + lane] = (uint16_t)ent;
    c = nx;
    const int32_t nlo = c / FR_CH;
    if (nlo == lo + 1) {
      // chunk lo's slot takes chunk lo + 2 (prefetched); prefetch lo + 3
      if (lo + 2 <= FR_KMAX) fr_store(ring, lo + 2, lane, pa, pb);
      lo = nlo;
      if (lo + 2 <= FR_KMAX) fr_load(buf, n, ts, lo + 2, lane, pa, pb);
    } else {
      // a frame longer than a chunk: restage around the landing point
      lo = nlo;
      uint4 a0, b0, a1, b1;
      fr_load(buf, n, ts, lo, lane, a0, b0);
      fr_load(buf, n, ts, lo + 1, lane, a1, b1);
      fr_store(ring, lo, lane, a0, b0);
      fr_store(ring, lo + 1, lane, a1, b1);
      if (lo + 2 <= FR_KMAX) fr_load(buf, n, ts, lo + 2, lane, pa, pb);
    }
  }
  uint16_t fin;
  {
    const int32_t len = fr_len(ring, c);
    int32_t q = 0;
    fin = fe_hop_len(len, c, nrel, maxp32, q);
    if (!((fin & F0_TERM) && fin != F0_ESC)) {  // leaves the tile: a start
      ent = lane == (m & 63) ? (uint32_t)c : ent;
      ++m;
      if ((m & 63) == 0) L[m - 64 + lane] = (uint16_t)ent;
      send = ts + c + 4 + len;
    } else {
      const bool bad = (c + 4 <= nrel) && ((uint32_t)len > umax);
      send = TERM | (bad ? TBAD : 0) | (ts + c);
    }
  }
  if (lane < (m & 63)) L[(m & ~63) + lane] = (uint16_t)ent;
  if (lane == 0) rcount[t * FE_NSURV] = m;
  uint16_t fins[FE_NSURV] = {fin};
  const int64_t k = fe_patch_row(f0 + t * W, W, lane, fins, ts);
  return (send & TERM) ? k : send;
}

// Composition path: one wave per tile (blockIdx), host length.
__global__ __launch_bounds__(64) void fs_survivor_r(
    const uint8_t* __restrict__ buf, int64_t n, int64_t maxp, int32_t W,
    uint16_t* __restrict__ f0, const int32_t* __restrict__ surv,
    uint16_t* __restrict__ list, int32_t* __restrict__ rcount) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[FR_RING];
  const int64_t t = blockIdx.x;
  if (t * FS_S >= n) return;
  int64_t send;
  (void)fs_survive(buf, n, maxp, W, f0, surv, list, rcount, t, ring,
                   threadIdx.x, send);
}

// D'' fs_join: the tile's frame starts from its exact entry e*.  Every chain
// that reaches a survivor's tree passes through that survivor's hand-off
// position r0 = R[0] (merges into it all happened at positions <= r0), so
// walk from e* (uniform scalar loop, global memory, usually 0-5 hops) until
// one of the r0, then the rest is that R.  A chain that meets neither (bad
// frame, or survivors that were garbage chains) is simply walked to its end.
__global__ __launch_bounds__(256) void fs_join(
    const uint8_t* __restrict__ buf, int64_t n, int64_t maxp, int64_t tiles,
    const int64_t* __restrict__ ent, const uint16_t* __restrict__ list,
    const int32_t* __restrict__ rcount, uint16_t* __restrict__ pre,
    int32_t* __restrict__ npre_out, int64_t* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= tiles) return;
  const int64_t e = ent[t];
  if (e == NONE) {
    if (lane == 0) { counts[t] = 0; npre_out[t] = 0; }
    return;
  }
  const int64_t ts = t * FS_S;
  const int32_t te = (int32_t)(min(ts + FS_S, n) - ts);
  const int32_t nrel = (int32_t)min(n - ts, (int64_t)1 << 30);
  const int32_t maxp32 = (int32_t)min(maxp, (int64_t)1 << 30);
  const int32_t m0 = __builtin_amdgcn_readfirstlane(rcount[t * FE_NSURV]);
  int32_t r0 = m0 > 0 ? __builtin_amdgcn_readfirstlane(
                            (int32_t)list[(t * FE_NSURV) * FS_LMAX]) : -1;
  int32_t m1 = 0, r1 = -1;
  if constexpr (FE_NSURV > 1) {
    m1 = __builtin_amdgcn_readfirstlane(rcount[t * FE_NSURV + 1]);
    r1 = m1 > 0 ? __builtin_amdgcn_readfirstlane(
                      (int32_t)list[(t * FE_NSURV + 1) * FS_LMAX]) : -1;
  }
  int32_t c = __builtin_amdgcn_readfirstlane((int32_t)(e - ts));
  int32_t np = 0;
  int32_t use = -1;
  uint16_t* P = pre + t * FS_LMAX;
  while (c < te) {
    if (c == r0) { use = 0; break; }
    if (c == r1) { use = 1; break; }
    if (c > r0) r0 = -1;                   // not in that survivor's tree
    if (c > r1) r1 = -1;
    if (c + 4 > nrel) break;               // partial length at the end
    const int32_t len = __builtin_amdgcn_readfirstlane(ld_be32(buf + ts + c));
    const int32_t nx = c + 4 + len;
    if ((len < 0) | (len > maxp32) | (nx > nrel)) break;
    if (lane == 0) P[np] = (uint16_t)c;
    ++np;
    c = nx;
  }
  if (lane == 0) {
    // npre: prefix length | the survivor slot whose R follows (-1: none)
    npre_out[t] = np | ((use + 1) << 28);
    counts[t] = np + (use == 0 ? m0 : (use == 1 ? m1 : 0));
  }
}

// E'' list -> (body offset, length): prefix from fs_join, then that R.
__global__ __launch_bounds__(256) void fs_write_join(
    const uint8_t* __restrict__ buf, int64_t tiles,
    const uint16_t* __restrict__ pre, const int32_t* __restrict__ npre,
    const uint16_t* __restrict__ list, const int64_t* __restrict__ counts,
    const int64_t* __restrict__ base, int64_t* __restrict__ foff,
    int32_t* __restrict__ flen, int64_t cap, int64_t* __restrict__ result) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= tiles) return;
  const int lane = threadIdx.x & 63;
  const int64_t cnt = counts[t];
  const int32_t pk = npre[t];
  const int32_t np = pk & 0x0FFFFFFF;
  const int32_t use = (pk >> 28) - 1;
  const int64_t b = base[t];
  const int64_t ts = t * FS_S;
  const uint16_t* Pp = pre + t * FS_LMAX;
  const uint16_t* R = list + (t * FE_NSURV + (use < 0 ? 0 : use)) * FS_LMAX;
  for (int64_t k = lane; k < cnt; k += 64) {
    const int64_t P = ts + (k < np ? Pp[k] : R[k - np]);
    const int64_t idx = b + k;
    if (idx < cap) {
      foff[idx] = P + 4;
      flen[idx] = ld_be32(buf + P);
    } else {
      result[3] = 1;
    }
  }
}

// ---- chain resolution (default): fs_tile, fs_link, fs_rows ------------------
// Replaces composition / push-down / join / count scan / write (13-15
// launches per scan) with three:
//
//  fs_tile   one wave per tile, tiles in order from an atomic counter: the
//            survivor walk (fs_survive), then publish the tile's speculated
//            exit X[t] and take the tile before's X[t-1] as this tile's
//            entry (a one-step wait: that tile started earlier and does the
//            same work).  The entry is exact unless a frame longer than the
//            window ends in the tile before, or its chain is not the
//            survivor's.  Walk from the entry through a 1 KiB LDS window
//            until the chain meets the survivor's recorded path (merge-walk
//            against the sorted list), leaves the tile, or ends in a
//            terminal; record (entry used, exit, count, walked starts).
//  fs_link   one workgroup: every link is checked in parallel (tile k's
//            entry must be tile k-1's exit); the leftmost broken links are
//            repaired by re-walking those tiles from the exact exit (wave 0,
//            serial, rare), then a block scan of the counts up to the first
//            terminal gives every tile its row base and result[0..3].
//  fs_rows   one wave per tile writes its (body offset, length) rows.
//
// (A single-pass decoupled look-back was tried first: with every tile of a
// 200 MB stream resident at once, each tile looked back across all the
// tiles before it, 64 per round trip: ~100 us per scan.)
constexpr int FC_WIN = 1024;                 // staged walk window (bytes)
constexpr int64_t FC_MAXP = (int64_t)1 << 24;
constexpr int FL_T = 1024;                   // fs_link threads

ZK_DEV uint64_t lb_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
ZK_DEV void lb_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
ZK_DEV int64_t ld_agent(const int64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
ZK_DEV void st_agent(int64_t* p, int64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Chain statistics after the tile counter: [1] tiles without a speculated
// entry, [2] tiles re-walked by fs_link, [3] fs_link repair rounds
// (zk_frame_scan_stats reads them).
ZK_DEV void fc_stat(uint64_t* stats, int k, uint32_t v) {
  __hip_atomic_fetch_add((uint32_t*)&stats[k], v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}

struct FcWalk {
  int64_t exit;      // exit position, or the terminal's position
  int32_t cnt;       // frame starts in the tile on the chain
  int32_t np;        // of which walked here (pre[0..np))
  int32_t js;        // survivor list index the rest starts at (-1: none)
  bool term, bad;
};

// per-tile record: meta = cnt | np << 13 | (js + 1) << 26 | term << 39 |
// bad << 40; entry = the entry used (-1: none, the tile before had no
// speculated exit)
ZK_DEV int64_t fc_meta(const FcWalk& w) {
  return (int64_t)w.cnt | ((int64_t)w.np << 13) | ((int64_t)(w.js + 1) << 26) |
         ((int64_t)w.term << 39) | ((int64_t)w.bad << 40);
}
ZK_DEV int32_t m_cnt(int64_t m) { return (int32_t)(m & 0x1FFF); }
ZK_DEV int32_t m_np(int64_t m) { return (int32_t)((m >> 13) & 0x1FFF); }
ZK_DEV int32_t m_js(int64_t m) { return (int32_t)((m >> 26) & 0x1FFF) - 1; }
ZK_DEV bool m_term(int64_t m) { return (m >> 39) & 1; }
ZK_DEV bool m_bad(int64_t m) { return (m >> 40) & 1; }

// Stage [wb, wb + FC_WIN) (zero past n) into the wave's window.
ZK_DEV void fc_stage(const uint8_t* __restrict__ buf, int64_t n, int64_t wb,
                     uint8_t* win, int lane) {
  const int64_t g = wb + 16 * lane;
  uint4 v = make_uint4(0, 0, 0, 0);
  if (g + 16 <= n) {
    __builtin_memcpy(&v, buf + g, 16);
  } else if (g < n) {
    uint8_t* b = (uint8_t*)&v;
    for (int k = 0; k < 16; ++k) b[k] = g + k < n ? buf[g + k] : 0;
  }
  *(uint4*)(win + 16 * lane) = v;
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Walk tile [ts, ts + S)'s chain from E (one wave, wave-uniform control).
// Frame starts walked before meeting the survivor's path L[0..m0) go to
// pre[] (tile-relative, written by lane 0).
ZK_DEV FcWalk fc_walk(const uint8_t* __restrict__ buf, int64_t n,
                      int64_t maxp, int64_t ts, int64_t E, const uint16_t* L,
                      int32_t m0, int64_t send, uint8_t* win, uint16_t* pre,
                      int lane) {
  FcWalk r{E, 0, 0, -1, false, false};
  const int64_t tend = ts + FS_S;
  int64_t c = E;
  int64_t wb = -(int64_t)FC_WIN;
  int32_t lb = 0;                             // survivor list window base
  uint32_t lv = lane < m0 ? (uint32_t)L[lane] : 0xFFFFFFFFu;
  int32_t np = 0;
  for (;;) {
    if (c >= tend) { r.exit = c; break; }
    if (c >= n) { r.exit = n; break; }        // the stream ends cleanly
    const uint32_t crel = (uint32_t)(c - ts);
    if (m0 > 0) {
      // merge-walk against the sorted survivor list
      while (lb + 64 < m0 &&
             crel > (uint32_t)__builtin_amdgcn_readlane((int)lv, 63)) {
        lb += 64;
        lv = lb + lane < m0 ? (uint32_t)L[lb + lane] : 0xFFFFFFFFu;
      }
      const uint64_t hit = __ballot(lv == crel);
      if (hit) {
        r.js = lb + (int32_t)__builtin_ctzll(hit);
        break;
      }
    }
    if (c + 4 > n) { r.exit = c; r.term = true; break; }
    if (c < wb || c + 8 > wb + FC_WIN) {
      wb = c & ~(int64_t)15;
      fc_stage(buf, n, wb, win, lane);
    }
    const int32_t o = (int32_t)(c - wb);
    const uint32_t raw = ((uint32_t)win[o] << 24) | ((uint32_t)win[o + 1] << 16) |
                         ((uint32_t)win[o + 2] << 8) | (uint32_t)win[o + 3];
    const int32_t len = __builtin_amdgcn_readfirstlane((int32_t)raw);
    if (len < 0 || (int64_t)len > maxp) {
      r.exit = c; r.term = true; r.bad = true; break;
    }
    const int64_t nx = c + 4 + len;
    if (nx > n) { r.exit = c; r.term = true; break; }
    if (lane == 0) pre[np] = (uint16_t)crel;
    ++np;
    c = nx;
  }
  r.np = np;
  r.cnt = np;
  if (r.js >= 0) {
    r.cnt = np + (m0 - r.js);
    if (send & TERM) {
      const int64_t q = send & ~(TERM | TBAD);
      if (q >= n && !(send & TBAD)) {
        r.exit = n;                           // clean end of the stream
      } else {
        r.exit = q; r.term = true; r.bad = (send & TBAD) != 0;
      }
    } else {
      r.exit = send;
    }
  }
  return r;
}

__global__ __launch_bounds__(64) void fs_tile(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ n_dev,
    int64_t n_cap, int64_t maxp, int32_t W, uint16_t* __restrict__ f0,
    const int32_t* __restrict__ surv, uint16_t* __restrict__ list,
    int32_t* __restrict__ rcount, int64_t* __restrict__ sx, uint64_t* lbw,
    uint16_t* __restrict__ pre, int64_t* __restrict__ rec_entry,
    int64_t* __restrict__ rec_exit, int64_t* __restrict__ rec_meta,
    int64_t* __restrict__ dbg) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[FR_RING];
  __shared__ __attribute__((aligned(16))) uint8_t win[FC_WIN + 16];
  const int64_t t_0 = dbg ? wall_clock64() : 0;
  const int lane = threadIdx.x;
  const int64_t n = stream_len(n_dev, n_cap);
  const int64_t ntiles = (n + FS_S - 1) / FS_S;
  uint64_t* stats = &lbw[2 * (int64_t)gridDim.x];
  uint32_t tid = 0;
  if (lane == 0)
    tid = __hip_atomic_fetch_add((uint32_t*)stats, 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
  const int64_t t = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)tid);
  if (t >= ntiles) return;
  const int64_t ts = t * FS_S;
  int64_t send;
  const int64_t cxt = fs_survive(buf, n, maxp, W, f0, surv, list, rcount, t,
                                 ring, lane, send);
  if (lane == 0) {
    sx[t] = send;
    lb_store(&lbw[2 * t], (uint64_t)(cxt + 2));      // X[t] (0 = not yet)
  }
  const int64_t t_1 = dbg ? wall_clock64() : 0;
  int64_t E = 0;
  bool none = false;
  if (t > 0) {
    uint64_t x;
    for (;;) {                                // tile t-1 is running or done
      x = lb_load(&lbw[2 * (t - 1)]);
      if (x != 0) break;
      __builtin_amdgcn_s_sleep(1);
    }
    E = (int64_t)x - 2;
    none = E < 0;
  }
  const int64_t t_2 = dbg ? wall_clock64() : 0;
  FcWalk w{E, 0, 0, -1, false, false};
  if (!none) {
    // this wave wrote list[t] and rcount[t] itself (every lane rereads
    // only the list entries it stored)
    const int32_t m0 = __builtin_amdgcn_readfirstlane(rcount[t]);
    w = fc_walk(buf, n, maxp, ts, E, list + t * FS_LMAX, m0, send, win,
                pre + t * FS_LMAX, lane);
  } else if (lane == 0) {
    fc_stat(stats, 1, 1);
  }
  if (lane == 0) {
    rec_entry[t] = none ? -1 : E;
    rec_exit[t] = w.exit;
    rec_meta[t] = fc_meta(w);
    if (dbg) {
      dbg[6 * t + 0] = t_0;
      dbg[6 * t + 1] = t_1;
      dbg[6 * t + 2] = t_2;
      dbg[6 * t + 3] = wall_clock64();
      dbg[6 * t + 4] = w.np;
      dbg[6 * t + 5] = w.js;
    }
  }
}

__global__ __launch_bounds__(FL_T) void fs_link(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ n_dev,
    int64_t n_cap, int64_t maxp, const int64_t* __restrict__ sx,
    const uint16_t* __restrict__ list, const int32_t* __restrict__ rcount,
    uint16_t* pre, int64_t* rec_entry, int64_t* rec_exit, int64_t* rec_meta,
    int64_t* __restrict__ base, int64_t cap, int64_t* __restrict__ result,
    uint64_t* stats) {
  __shared__ __attribute__((aligned(16))) uint8_t win[FC_WIN + 16];
  __shared__ int64_t red[2 * (FL_T / 64) + 2];
  __shared__ int64_t s_next;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t n = stream_len(n_dev, n_cap);
  const int64_t ntiles = (n + FS_S - 1) / FS_S;
  if (ntiles == 0) return;                    // result zeroed by fs_frontier
  const int64_t INF = INT64_MAX;
  int64_t from = 1, ft = INF;
  for (;;) {
    // leftmost terminal, and leftmost broken link at or after `from` (tile
    // k's entry must be tile k-1's exit; links before `from` hold)
    int64_t fb = INF, fterm = INF;
    for (int64_t k = tid; k < ntiles; k += FL_T) {
      const int64_t mk = ld_agent(&rec_meta[k]);
      if (m_term(mk)) {
        fterm = min(fterm, k);
      } else if (k + 1 < ntiles && k + 1 >= from) {
        const int64_t e = ld_agent(&rec_entry[k + 1]);
        if (e < 0 || e != ld_agent(&rec_exit[k])) fb = min(fb, k + 1);
      }
    }
    for (int d = 32; d >= 1; d >>= 1) {
      fb = min(fb, (int64_t)__shfl_xor(fb, d, 64));
      fterm = min(fterm, (int64_t)__shfl_xor(fterm, d, 64));
    }
    if (lane == 0) { red[wv] = fb; red[FL_T / 64 + wv] = fterm; }
    __syncthreads();
    fb = INF;
    fterm = INF;
    for (int j = 0; j < FL_T / 64; ++j) {
      fb = min(fb, red[j]);
      fterm = min(fterm, red[FL_T / 64 + j]);
    }
    __syncthreads();
    if (fb == INF || fb > fterm) {            // every live link holds
      ft = fterm;
      break;
    }
    // repair: re-walk tiles from fb while their links stay broken
    if (wv == 0) {
      int64_t k = fb;
      uint32_t walked = 0;
      for (;;) {
        const int64_t E = ld_agent(&rec_exit[k - 1]);
        const int32_t m0 = __builtin_amdgcn_readfirstlane(rcount[k]);
        const FcWalk w = fc_walk(buf, n, maxp, k * FS_S, E,
                                 list + k * FS_LMAX, m0, sx[k], win,
                                 pre + k * FS_LMAX, lane);
        ++walked;
        if (lane == 0) {
          st_agent(&rec_entry[k], E);
          st_agent(&rec_exit[k], w.exit);
          st_agent(&rec_meta[k], fc_meta(w));
        }
        ++k;
        if (w.term || k >= ntiles) break;
        if (ld_agent(&rec_entry[k]) == w.exit) break;   // link k holds
      }
      if (lane == 0) {
        s_next = k;
        fc_stat(stats, 2, walked);
        fc_stat(stats, 3, 1);
      }
    }
    __syncthreads();
    from = s_next;
  }
  // exclusive scan of the counts of tiles 0..ft; tiles after ft are dead
  const int64_t last = ft == INF ? ntiles - 1 : ft;
  const int64_t per = (last + 1 + FL_T - 1) / FL_T;
  const int64_t k0 = (int64_t)tid * per;
  const int64_t k1 = min(k0 + per, last + 1);
  int64_t sum = 0;
  for (int64_t k = k0; k < k1; ++k) sum += m_cnt(ld_agent(&rec_meta[k]));
  int64_t tot;
  int64_t run = block_excl_scan(sum, red, &tot);
  for (int64_t k = k0; k < k1; ++k) {
    base[k] = run;
    run += m_cnt(ld_agent(&rec_meta[k]));
  }
  for (int64_t k = last + 1 + tid; k < ntiles; k += FL_T) base[k] = -1;
  if (tid == 0) {
    result[0] = tot;
    result[3] = tot > cap ? 1 : 0;
    if (ft == INF) {
      result[1] = n;
      result[2] = 0;
    } else {
      result[1] = ld_agent(&rec_exit[ft]);
      result[2] = m_bad(ld_agent(&rec_meta[ft])) ? 1 : 0;
    }
  }
}

// (body offset, length) rows: one wave per tile, 4 tiles per block.
__global__ __launch_bounds__(256) void fs_rows(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ n_dev,
    int64_t n_cap, const uint16_t* __restrict__ list,
    const uint16_t* __restrict__ pre, const int64_t* __restrict__ rec_meta,
    const int64_t* __restrict__ base, int64_t* __restrict__ foff,
    int32_t* __restrict__ flen, int64_t cap) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t n = stream_len(n_dev, n_cap);
  if (t * FS_S >= n) return;
  const int64_t b = base[t];
  if (b < 0) return;
  const int64_t m = rec_meta[t];
  const int32_t cnt = m_cnt(m), np = m_np(m), js = m_js(m);
  const int64_t ts = t * FS_S;
  const uint16_t* P = pre + t * FS_LMAX;
  const uint16_t* R = list + t * FS_LMAX + (js < 0 ? 0 : js);
  for (int32_t k = lane; k < cnt; k += 64) {
    const int64_t pos = ts + (k < np ? P[k] : R[k - np]);
    const int64_t idx = b + k;
    if (idx < cap) {
      foff[idx] = pos + 4;
      flen[idx] = ld_be32(buf + pos);
    }
  }
}

struct FsPlan {
  int levels;
  int64_t units[FS_MAXL];
  int64_t usize[FS_MAXL];
  size_t off_f0, off_fl[FS_MAXL], off_ent[FS_MAXL], off_cnt, off_base,
      off_scan, off_list, off_pre, off_surv, off_rcnt, off_npre, off_cx,
      off_sx, off_lbw, off_rent, off_rexit, off_rmeta, total;
};

// Workspace of a scan over a buffer of n bytes.  The one-pass chain needs
// f0, the survivor lists and 40 bytes per tile; the composition path (A/B)
// its level tables, entries and count scan on top.
static FsPlan fs_plan(int64_t n, int64_t W) {
  FsPlan p{};
  const int64_t tiles = n > 0 ? (n + FS_S - 1) / FS_S : 1;
  p.units[0] = tiles;
  p.usize[0] = FS_S;
  p.levels = 1;
  while (p.units[p.levels - 1] > FS_TOPMAX && p.levels < FS_MAXL) {
    const int l = p.levels;
    p.usize[l] = p.usize[l - 1] * FS_G;
    p.units[l] = (p.units[l - 1] + FS_G - 1) / FS_G;
    p.levels++;
  }
  size_t o = 0;
  auto take = [&](size_t bytes) { size_t r = o; o += (bytes + 255) & ~(size_t)255; return r; };
  p.off_f0 = take((size_t)tiles * W * 2);
  p.off_list = take((size_t)tiles * FE_NSURV * FS_LMAX * 2);
  p.off_surv = take((size_t)tiles * FE_NSURV * 4);
  p.off_rcnt = take((size_t)tiles * FE_NSURV * 4);
  p.off_cx = take((size_t)tiles * 8);
  p.off_sx = take((size_t)tiles * 8);
  p.off_lbw = take((size_t)(2 * tiles + 4) * 8);
  p.off_rent = take((size_t)tiles * 8);
  p.off_rexit = take((size_t)tiles * 8);
  p.off_rmeta = take((size_t)tiles * 8);
  p.off_pre = take((size_t)tiles * FS_LMAX * 2);
  p.off_base = take((size_t)tiles * 8);
  for (int l = 1; l < p.levels; ++l)
    p.off_fl[l] = take((size_t)p.units[l] * W * 8);
  for (int l = 0; l < p.levels; ++l) p.off_ent[l] = take((size_t)p.units[l] * 8);
  p.off_cnt = take((size_t)tiles * 8);
  p.off_scan = take((size_t)zk_scan_workspace(tiles) * 8);
  p.off_npre = take((size_t)tiles * 4);
  p.total = o;
  return p;
}

static int fs_window(int32_t window) {
  return window <= 256 ? 256 : window <= 512 ? 512
       : window <= 1024 ? 1024 : (int)FS_W;
}

static void fs_launch_frontier(int W, int64_t tiles, const uint8_t* buf,
                               const int64_t* n_dev, int64_t n_cap,
                               int64_t maxp, uint16_t* f0, int32_t* surv,
                               uint64_t* lbw, int64_t* result,
                               hipStream_t st) {
  switch (W) {
    case 256:
      fs_frontier<256><<<(unsigned)tiles, FE_T, fe_lds(256), st>>>(
          buf, n_dev, n_cap, maxp, f0, surv, lbw, result);
      break;
    case 512:
      fs_frontier<512><<<(unsigned)tiles, FE_T, fe_lds(512), st>>>(
          buf, n_dev, n_cap, maxp, f0, surv, lbw, result);
      break;
    case 1024:
      fs_frontier<1024><<<(unsigned)tiles, FE_T, fe_lds(1024), st>>>(
          buf, n_dev, n_cap, maxp, f0, surv, lbw, result);
      break;
    default:
      fs_frontier<(int)FS_W><<<(unsigned)tiles, FE_T, fe_lds((int)FS_W),
                               st>>>(buf, n_dev, n_cap, maxp, f0, surv, lbw,
                                     result);
  }
}

// The composition path (ZKMI_FS_SCAN=compose, A/B only): host length n.
static int fs_scan_compose(const uint8_t* buf, int64_t n, int64_t maxp,
                           uint8_t* ws, int64_t ws_bytes, int64_t* foff,
                           int32_t* flen, int64_t cap, int64_t* result, int W,
                           hipStream_t st) {
  FsPlan p = fs_plan(n, W);
  if ((int64_t)p.total > ws_bytes) return -1;
  (void)hipMemsetAsync(result, 0, 4 * sizeof(int64_t), st);
  if (n <= 0) return 0;
  FsCtx c{};
  c.buf = buf;
  c.n = n;
  c.maxp = maxp;
  c.W = W;
  c.levels = p.levels;
  for (int l = 0; l < p.levels; ++l) {
    c.units[l] = p.units[l];
    c.usize[l] = p.usize[l];
    c.ent[l] = (int64_t*)(ws + p.off_ent[l]);
    if (l > 0) c.fl[l] = (int64_t*)(ws + p.off_fl[l]);
  }
  c.f0 = (const uint16_t*)(ws + p.off_f0);
  const int64_t tiles = p.units[0];
  uint16_t* f0w = (uint16_t*)(ws + p.off_f0);
  int64_t* cnt = (int64_t*)(ws + p.off_cnt);
  int64_t* base = (int64_t*)(ws + p.off_base);
  uint16_t* list = (uint16_t*)(ws + p.off_list);
  uint16_t* pre = (uint16_t*)(ws + p.off_pre);
  int32_t* surv = (int32_t*)(ws + p.off_surv);
  int32_t* rcnt = (int32_t*)(ws + p.off_rcnt);
  int32_t* npre = (int32_t*)(ws + p.off_npre);
  fs_launch_frontier(W, tiles, buf, nullptr, n, maxp, f0w, surv, nullptr,
                     nullptr, st);
  ZK_LAUNCH_CHECK();
  fs_survivor_r<<<(unsigned)tiles, 64, 0, st>>>(buf, n, maxp, W, f0w, surv,
                                               list, rcnt);
  ZK_LAUNCH_CHECK();
  for (int l = 0; l + 1 < p.levels; ++l) {
    const size_t sb = fs_stage_bytes(l, W);
    if (sb <= FS_STAGE_MAX)
      fs_compose_staged<<<(unsigned)p.units[l + 1], min(W, FS_T), sb, st>>>(
          c, l);
    else
      fs_compose<<<(unsigned)p.units[l + 1], min(W, FS_T), 0, st>>>(c, l);
    ZK_LAUNCH_CHECK();
  }
  fs_top<<<1, 64, 0, st>>>(c, result);
  ZK_LAUNCH_CHECK();
  for (int l = p.levels - 2; l >= 0; --l) {
    const int64_t np = p.units[l + 1];
    const size_t sb = fs_stage_bytes(l, W);
    if (sb <= FS_STAGE_MAX)
      fs_down_staged<<<(unsigned)np, 64, sb, st>>>(c, l);
    else
      fs_down<<<(unsigned)((np + 255) / 256), 256, 0, st>>>(c, l);
    ZK_LAUNCH_CHECK();
  }
  const unsigned wblocks = (unsigned)((tiles + 3) / 4);
  fs_join<<<wblocks, 256, 0, st>>>(buf, n, maxp, tiles, c.ent[0], list, rcnt,
                                   pre, npre, cnt);
  ZK_LAUNCH_CHECK();
  int rc = zk_scan_excl_i64(cnt, base, tiles, result + 0,
                            (int64_t*)(ws + p.off_scan), st);
  if (rc) return rc;
  fs_write_join<<<wblocks, 256, 0, st>>>(buf, tiles, pre, npre, list, cnt,
                                         base, foff, flen, cap, result);
  ZK_LAUNCH_CHECK();
  return 0;
}

}  // namespace zk

extern "C" {

// Sized for the largest window (FS_W), an upper bound for any window.
int64_t zk_frame_scan_workspace(int64_t n) {
  return (int64_t)zk::fs_plan(n, zk::FS_W).total;
}

// K1 over buf[0, n) with n = min(*n_dev, n_cap) read ON THE DEVICE (n_dev
// null: n = n_cap).  Four launches: fs_frontier, fs_tile, fs_link, fs_rows;
// the grid covers n_cap and tiles past n return at once, so a producer's
// device byte count (an encoder's `total`) is scanned with no host read and
// no byte past it is touched.
//
// result (device int64[4]): [0] frames found, [1] stop offset (consumed
// bytes; start of the carry or of the bad frame), [2] 1 if the stop is a
// BAD_LENGTH frame, [3] 1 if the frame table overflowed `cap` (rows past
// cap are dropped).
//
// `window` (256 / 512 / 1024 / 2048 bytes) is the fast-path entry window per
// 16 KiB tile: a chain can only enter a tile inside it when frames are <=
// window bytes, so the frontier walks `window` speculative entry points per
// tile.  Longer frames stay exact (their tiles' entries come from the exact
// look-back instead of a constant exit), so the window is a performance
// hint: the smallest one covering the stream's usual frame size makes the
// scan cheapest.  maxp must be <= 16 MiB (the protocol's frame limit).
// ZKMI_FS_DBG=1: fs_tile writes per-tile timestamps (start, survivor done,
// entry known, walk done) and the walk's (np, js) into a debug buffer
// (zk_frame_scan_dbg copies it out).  Diagnostics only.
static int64_t* g_dbg = nullptr;
static int64_t g_dbg_tiles = 0;
static int64_t* fs_dbg_buf(int64_t tiles) {
  static int on = -1;
  if (on < 0) on = getenv("ZKMI_FS_DBG") != nullptr;
  if (!on) return nullptr;
  if (tiles > g_dbg_tiles) {
    if (g_dbg) (void)hipFree(g_dbg);
    if (hipMalloc(&g_dbg, tiles * 6 * 8) != hipSuccess) return nullptr;
    g_dbg_tiles = tiles;
  }
  return g_dbg;
}

int zk_frame_scan_dbg(int64_t* host, int64_t tiles) {
  if (!g_dbg || tiles > g_dbg_tiles) return -1;
  return hipMemcpy(host, g_dbg, tiles * 6 * 8, hipMemcpyDeviceToHost) ==
                 hipSuccess ? 0 : -1;
}

int zk_frame_scan3(const uint8_t* buf, const int64_t* n_dev, int64_t n_cap,
                   int64_t maxp, uint8_t* ws, int64_t ws_bytes, int64_t* foff,
                   int32_t* flen, int64_t cap, int64_t* result, int32_t window,
                   hipStream_t st) {
  using namespace zk;
  const int W = fs_window(window);
  if (maxp > FC_MAXP || maxp < 0) return -3;
  // ZKMI_FS_SCAN=compose: the round-1 composition path (host length only)
  static int mode = -1;
  if (mode < 0) {
    const char* m = getenv("ZKMI_FS_SCAN");
    mode = (m && m[0] == 'c') ? 1 : 0;
  }
  if (mode == 1 && n_dev == nullptr)
    return fs_scan_compose(buf, n_cap, maxp, ws, ws_bytes, foff, flen, cap,
                           result, W, st);
  FsPlan p = fs_plan(n_cap, W);
  if ((int64_t)p.total > ws_bytes) return -1;
  const int64_t tiles = p.units[0];
  uint16_t* f0w = (uint16_t*)(ws + p.off_f0);
  uint16_t* list = (uint16_t*)(ws + p.off_list);
  int32_t* surv = (int32_t*)(ws + p.off_surv);
  int32_t* rcnt = (int32_t*)(ws + p.off_rcnt);
  int64_t* cx = (int64_t*)(ws + p.off_cx);
  int64_t* sx = (int64_t*)(ws + p.off_sx);
  uint64_t* lbw = (uint64_t*)(ws + p.off_lbw);
  uint16_t* pre = (uint16_t*)(ws + p.off_pre);
  int64_t* rent = (int64_t*)(ws + p.off_rent);
  int64_t* rexit = (int64_t*)(ws + p.off_rexit);
  int64_t* rmeta = (int64_t*)(ws + p.off_rmeta);
  int64_t* base = (int64_t*)(ws + p.off_base);
  (void)cx;
  fs_launch_frontier(W, tiles, buf, n_dev, n_cap, maxp, f0w, surv, lbw,
                     result, st);
  ZK_LAUNCH_CHECK();
  fs_tile<<<(unsigned)tiles, 64, 0, st>>>(buf, n_dev, n_cap, maxp, W, f0w,
                                         surv, list, rcnt, sx, lbw, pre, rent,
                                         rexit, rmeta, fs_dbg_buf(tiles));
  ZK_LAUNCH_CHECK();
  fs_link<<<1, FL_T, 0, st>>>(buf, n_dev, n_cap, maxp, sx, list, rcnt, pre,
                              rent, rexit, rmeta, base, cap, result,
                              lbw + 2 * tiles);
  ZK_LAUNCH_CHECK();
  fs_rows<<<(unsigned)((tiles + 3) / 4), 256, 0, st>>>(
      buf, n_dev, n_cap, list, pre, rmeta, base, foff, flen, cap);
  ZK_LAUNCH_CHECK();
  return 0;
}

// Copy the chain statistics of the last scan of workspace `ws` over a
// buffer of n_cap bytes (window W) into out3 (host): tiles without a
// speculated entry, tiles re-walked, repair rounds.
int zk_frame_scan_stats(const uint8_t* ws, int64_t n_cap, int32_t window,
                        uint32_t* out3, hipStream_t st) {
  using namespace zk;
  FsPlan p = fs_plan(n_cap, fs_window(window));
  const uint64_t* lbw = (const uint64_t*)(ws + p.off_lbw);
  for (int k = 0; k < 3; ++k)
    if (hipMemcpyAsync(out3 + k, lbw + 2 * p.units[0] + 1 + k, 4,
                       hipMemcpyDeviceToHost, st) != hipSuccess)
      return -1;
  return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
}

int zk_frame_scan2(const uint8_t* buf, int64_t n, int64_t maxp, uint8_t* ws,
                   int64_t ws_bytes, int64_t* foff, int32_t* flen, int64_t cap,
                   int64_t* result, int32_t window, hipStream_t st) {
  return zk_frame_scan3(buf, nullptr, n, maxp, ws, ws_bytes, foff, flen, cap,
                        result, window, st);
}

int zk_frame_scan(const uint8_t* buf, int64_t n, int64_t maxp, uint8_t* ws,
                  int64_t ws_bytes, int64_t* foff, int32_t* flen, int64_t cap,
                  int64_t* result, hipStream_t st) {
  return zk_frame_scan3(buf, nullptr, n, maxp, ws, ws_bytes, foff, flen, cap,
                        result, (int32_t)zk::FS_W, st);
}

}  // extern "C"

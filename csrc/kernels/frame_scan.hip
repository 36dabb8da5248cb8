// K1 — parallel length-prefixed frame scan.
//
// Reference: ZKDecodeStream._transform (lib/zk-streams.js:39-65) walks the
// i32-BE length chain one frame at a time and memmoves the remainder per
// packet (O(bytes x packets)).  The chain is inherently
// sequential; we make it parallel without speculation errors:
//
//  A  per-tile exit table f0[tile][e] for the W window entry points e (the
//     only places a chain can enter a tile when frames are <= W bytes):
//     fs_frontier + fs_survivor (default; merging frontier walk, see below)
//     or fs_exits (ZKMI_FS_SCAN=jump|double; pointer jumping over every
//     position of the tile):
//     fs_exits   one workgroup per 16 KiB tile: build next(p) = p + 4 +
//                be32(p) for EVERY byte position and pointer-jump (in place,
//                racy but monotone) until each position maps to the first
//                chain position outside the tile or to a terminal.
//  B  fs_compose hierarchical function composition: a level-(l+1) unit is 16
//                level-l units; for each window entry point, walk the 16
//                sub-unit functions.  Log-depth, O(W) work per unit.  The 16
//                child tables are staged in LDS first (fs_compose_staged).
//  C  fs_top/fs_down  serial walk over the (few) top units from the stream
//                start, then push the exact entry position down to every tile
//                (fs_down_staged: one wave per parent, children in LDS).
//  D  frame starts per tile from its exact entry: fs_join (default: walk from
//     the entry to the survivor's hand-off point, then reuse the survivor's
//     recorded path), fs_walk (jump: wave-uniform walk of the staged tile) or
//     fs_mark (double: doubling marks on the full tile + bitmap).
//  E  scan of counts (scan.hip) + fs_write_join / fs_write_list / fs_write:
//     frame starts -> (body_off, len) table.
//
// Frames longer than W (2 KiB) fall back to walking the byte chain in global
// memory for the tile they land in; results stay exact.  BAD_LENGTH is
// reported at the exact frame (result[1] = its offset, result[2] = 1), the
// consumed prefix ends at the last complete frame, and a partial trailing
// frame is left for the next call (carry), like the reference's buffer.
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

// next() of every tile position relative to the tile (>= S: leaves tile;
// == p: terminal).
ZK_DEV int32_t next_rel(const uint8_t* sb, int64_t ts, int64_t n, int64_t maxp,
                        int32_t p) {
  const int64_t P = ts + p;
  if (P + 4 > n) return p;
  const uint32_t raw = ((uint32_t)sb[p] << 24) | ((uint32_t)sb[p + 1] << 16) |
                       ((uint32_t)sb[p + 2] << 8) | (uint32_t)sb[p + 3];
  const int32_t len = (int32_t)raw;
  if (len < 0 || (int64_t)len > maxp) return p;
  if (P + 4 + len > n) return p;
  const int64_t nx = (int64_t)p + 4 + len;
  return nx > 0x7FFFFFF0LL ? 0x7FFFFFF0 : (int32_t)nx;
}

constexpr int FS_PT = FS_S / FS_T;      // positions per thread (16)

// In-place pointer jumping over a uint16 successor table whose fixed points
// are the sinks.  Each thread batches its 16 gathers before any store so the
// LDS reads of one round are all in flight together (the compiler cannot
// reorder them across the aliasing stores itself).
//
// Real streams have few long chains: in a GET_DATA reply stream ~70 % of the
// positions are sinks from the start and only the true frame chain (~90
// positions per 16 KiB tile) needs more than 3 doublings.  So: 2 full rounds,
// then compact the still-moving positions into an LDS list and iterate only
// over it (full rounds again if the list would overflow).
constexpr int FS_LIST = 4096;            // compacted active-position capacity

ZK_DEV void jump_to_sinks(uint16_t* J, uint16_t* act, int64_t* red) {
  for (int it = 0; it < 2; ++it) {
    uint16_t v[FS_PT], w[FS_PT];
#pragma unroll
    for (int k = 0; k < FS_PT; ++k) v[k] = J[threadIdx.x + k * FS_T];
#pragma unroll
    for (int k = 0; k < FS_PT; ++k) w[k] = J[v[k]];
    int changed = 0;
#pragma unroll
    for (int k = 0; k < FS_PT; ++k) {
      if (w[k] != v[k]) { J[threadIdx.x + k * FS_T] = w[k]; changed = 1; }
    }
    if (!__syncthreads_or(changed)) return;
  }
  // compact positions that have not reached their sink
  uint16_t v[FS_PT];
  uint32_t mask = 0;
#pragma unroll
  for (int k = 0; k < FS_PT; ++k) v[k] = J[threadIdx.x + k * FS_T];
#pragma unroll
  for (int k = 0; k < FS_PT; ++k)
    if (J[v[k]] != v[k]) mask |= 1u << k;
  int64_t tot;
  int64_t o = block_excl_scan(__popc(mask), red, &tot);
  if (tot > FS_LIST) {
    for (int it = 0; it < 16; ++it) {
      uint16_t a[FS_PT], b[FS_PT];
#pragma unroll
      for (int k = 0; k < FS_PT; ++k) a[k] = J[threadIdx.x + k * FS_T];
#pragma unroll
      for (int k = 0; k < FS_PT; ++k) b[k] = J[a[k]];
      int changed = 0;
#pragma unroll
      for (int k = 0; k < FS_PT; ++k)
        if (b[k] != a[k]) { J[threadIdx.x + k * FS_T] = b[k]; changed = 1; }
      if (!__syncthreads_or(changed)) return;
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < FS_PT; ++k)
    if (mask & (1u << k)) act[o++] = (uint16_t)(threadIdx.x + k * FS_T);
  __syncthreads();
  const int cnt = (int)tot;
  for (int it = 0; it < 16; ++it) {
    int changed = 0;
    for (int i = threadIdx.x; i < cnt; i += FS_T) {
      const int p = act[i];
      const uint16_t a = J[p];
      const uint16_t b = J[a];
      if (b != a) { J[p] = b; changed = 1; }
    }
    if (!__syncthreads_or(changed)) return;
  }
}

// A: per-tile exits.  J[p] = in-tile successor, or p itself when p is a
// terminal or its frame leaves the tile (a sink).  After jumping, J[p] is
// the last in-tile chain element of p; its next() is the exit (or it is a
// terminal).  16-bit table: 32 KiB + 16 KiB staged bytes -> 3 blocks / CU.
__global__ __launch_bounds__(FS_T) void fs_exits(const uint8_t* __restrict__ buf,
                                                int64_t n, int64_t maxp,
                                                uint16_t* __restrict__ f0) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint16_t* J = (uint16_t*)smem;                     // [S]
  uint16_t* act = (uint16_t*)(smem + FS_S * 2);      // [FS_LIST]
  int64_t* red = (int64_t*)(smem + FS_S * 2 + FS_LIST * 2);
  const int64_t t = blockIdx.x;
  const int64_t ts = t * FS_S;
  // Each thread owns 16 contiguous positions: one 16-byte + one 4-byte
  // global load cover the 19 bytes their length prefixes span; the BE32 at
  // every byte offset is rebuilt with v_alignbyte (no LDS byte staging).
  {
    const int32_t p0 = threadIdx.x * FS_PT;
    const int64_t B = ts + p0;
    uint32_t w[5];
    if (B + 20 <= n) {
      uint4 v; __builtin_memcpy(&v, buf + B, 16);
      w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
      __builtin_memcpy(&w[4], buf + B + 16, 4);
    } else {
#pragma unroll
      for (int d = 0; d < 5; ++d) {
        uint32_t x = 0;
        for (int b = 0; b < 4; ++b) {
          const int64_t a = B + 4 * d + b;
          x |= (a < n ? (uint32_t)buf[a] : 0u) << (8 * b);
        }
        w[d] = x;
      }
    }
    uint16_t j[FS_PT];
#pragma unroll
    for (int k = 0; k < FS_PT; ++k) {
      const uint32_t le = __builtin_amdgcn_alignbyte(w[(k >> 2) + 1],
                                                     w[k >> 2], k & 3);
      const int32_t len = (int32_t)bswap32(le);
      const int64_t P = B + k;
      const bool ok = (P + 4 <= n) && len >= 0 && (int64_t)len <= maxp &&
                      P + 4 + len <= n;
      const int64_t nx = ok ? (int64_t)(p0 + k) + 4 + len : (int64_t)(p0 + k);
      j[k] = (uint16_t)(nx < FS_S ? nx : p0 + k);
    }
    *(uint4*)(J + p0) = *(uint4*)j;
    *(uint4*)(J + p0 + 8) = *(uint4*)(j + 8);
  }
  __syncthreads();
  jump_to_sinks(J, act, red);
  for (int32_t p = threadIdx.x; p < FS_W; p += FS_T) {
    const int32_t q = J[p];
    const int64_t Q = ts + q;
    uint16_t v = F0_TERM | (uint16_t)q;              // terminal by default
    if (Q + 4 <= n) {
      const int32_t len = ld_be32(buf + Q);
      if (len >= 0 && (int64_t)len <= maxp && Q + 4 + len <= n) {
        const int64_t x = (int64_t)q + 4 + len - FS_S;   // >= 0: leaves tile
        v = x < 0x4000 ? (uint16_t)x : F0_ESC;
      }
    }
    f0[t * FS_W + p] = v;
  }
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
template <int W>
__global__ __launch_bounds__(FE_T) void fs_frontier(
    const uint8_t* __restrict__ buf, int64_t n, int64_t maxp,
    uint16_t* __restrict__ f0, int32_t* __restrict__ surv) {
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
  const int64_t ts = t * FS_S;
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

// Mark the chain inside each tile from its entry; bitmap of frame starts.
__global__ __launch_bounds__(FS_T) void fs_mark(const uint8_t* __restrict__ buf,
                                               int64_t n, int64_t maxp,
                                               const int64_t* __restrict__ ent,
                                               uint32_t* __restrict__ bits,
                                               int64_t* __restrict__ counts) {
  // LDS: A, B (uint16 [S] each), mk (uint8 [S]); the staged bytes live in
  // B's space until A is built.  80 KiB -> 2 blocks / CU.  Each thread owns
  // 16 CONTIGUOUS positions so mk / A / B move as 16-byte LDS vectors.
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint16_t* A = (uint16_t*)smem;                       // [S]
  uint16_t* B = A + FS_S;                              // [S]
  uint8_t* mk = smem + FS_S * 4;                       // [S] bit0 mark, bit1 terminal
  uint8_t* sb = (uint8_t*)B;                           // [S + 16] (aliases B)
  const int64_t t = blockIdx.x;
  const int64_t ts = t * FS_S;
  const int64_t e = ent[t];
  uint32_t* tb = bits + t * (FS_S / 32);
  if (e == NONE) {
    for (int k = threadIdx.x; k < FS_S / 32; k += FS_T) tb[k] = 0;
    if (threadIdx.x == 0) counts[t] = 0;
    return;
  }
  const int32_t p0 = threadIdx.x * FS_PT;
  stage_tile<FS_T>(buf, n, ts, sb, threadIdx.x);
  __syncthreads();
  // A[p]: next within tile; S = leaves the tile; p itself = terminal.
  {
    uint16_t a[FS_PT];
    uint8_t m[FS_PT];
#pragma unroll
    for (int k = 0; k < FS_PT; ++k) {
      const int32_t p = p0 + k;
      const int32_t j = next_rel(sb, ts, n, maxp, p);
      a[k] = (uint16_t)(j >= FS_S ? FS_S : j);
      m[k] = (j == p) ? 2 : 0;
    }
    __syncthreads();                                   // sb (in B) is dead
#pragma unroll
    for (int k = 0; k < FS_PT; k += 8)
      *(uint4*)(A + p0 + k) = *(uint4*)(a + k);
    *(uint4*)(mk + p0) = *(uint4*)m;
  }
  __syncthreads();
  if (threadIdx.x == 0) mk[e - ts] |= 1;
  __syncthreads();
  for (int r = 0; r < 16; ++r) {
    // mark: every marked position marks its 2^r-th successor
    int added = 0;
    const uint4 mv = *(const uint4*)(mk + p0);
    const uint32_t mw[4] = {mv.x, mv.y, mv.z, mv.w};
    if ((mw[0] | mw[1] | mw[2] | mw[3]) & 0x01010101u) {
#pragma unroll
      for (int k = 0; k < FS_PT; ++k) {
        if ((mw[k >> 2] >> (8 * (k & 3))) & 1u) {
          const int32_t j = A[p0 + k];
          if (j < FS_S && j != p0 + k && !(mk[j] & 1)) {
            mk[j] |= 1;
            added = 1;
          }
        }
      }
    }
    if (!__syncthreads_or(added)) break;
    // jump: B = A o A
    uint16_t a[FS_PT], b[FS_PT];
    *(uint4*)a = *(const uint4*)(A + p0);
    *(uint4*)(a + 8) = *(const uint4*)(A + p0 + 8);
#pragma unroll
    for (int k = 0; k < FS_PT; ++k) {
      const int32_t j = a[k];
      b[k] = (j < FS_S && j != p0 + k) ? A[j] : (uint16_t)j;
    }
    *(uint4*)(B + p0) = *(uint4*)b;
    *(uint4*)(B + p0 + 8) = *(uint4*)(b + 8);
    __syncthreads();
    uint16_t* tmp = A; A = B; B = tmp;
  }
  // A frame starts at every marked position that is not a terminal.
  const uint4 mv = *(const uint4*)(mk + p0);
  const uint32_t mw[4] = {mv.x, mv.y, mv.z, mv.w};
  uint32_t half = 0;
#pragma unroll
  for (int k = 0; k < FS_PT; ++k)
    if (((mw[k >> 2] >> (8 * (k & 3))) & 3u) == 1u) half |= 1u << k;
  const uint32_t other = __shfl_xor(half, 1, 64);
  const uint32_t w = (threadIdx.x & 1) ? 0u : (half | (other << 16));
  if (!(threadIdx.x & 1)) tb[threadIdx.x >> 1] = w;
  __syncthreads();                                     // mk reads done
  int64_t* red = (int64_t*)mk;                         // reuse mk space
  int64_t tot;
  block_excl_scan((int64_t)__popc(w), red, &tot);
  if (threadIdx.x == 0) counts[t] = tot;
}

__global__ __launch_bounds__(256) void fs_write(const uint8_t* __restrict__ buf,
                                               const uint32_t* __restrict__ bits,
                                               const int64_t* __restrict__ base,
                                               int64_t* __restrict__ foff,
                                               int32_t* __restrict__ flen,
                                               int64_t cap,
                                               int64_t* __restrict__ result) {
  __shared__ int64_t red[256 / 64 + 1];
  const int64_t t = blockIdx.x;
  const int64_t ts = t * FS_S;
  const uint32_t* tb = bits + t * (FS_S / 32);
  // 512 words per tile, 2 per thread
  const int k0 = threadIdx.x * 2;
  const uint32_t w0 = tb[k0], w1 = tb[k0 + 1];
  int64_t tot;
  int64_t idx = base[t] + block_excl_scan(__popc(w0) + __popc(w1), red, &tot);
  for (int h = 0; h < 2; ++h) {
    uint32_t w = h ? w1 : w0;
    while (w) {
      const int b = __ffs(w) - 1;
      w &= w - 1;
      const int64_t P = ts + (int64_t)(k0 + h) * 32 + b;
      if (idx < cap) {
        foff[idx] = P + 4;
        flen[idx] = ld_be32(buf + P);
      } else {
        result[3] = 1;
      }
      ++idx;
    }
  }
}

// D' (default) — walk the chain of every tile from its entry, one lane per
// tile, straight from global memory.  Once the entries are known the walk is
// ~frames-per-tile dependent loads (the tile's lines come from L2 / the
// Infinity Cache, where the producer just wrote them), and all tiles walk
// concurrently, so the kernel is latency- not work-bound: it replaces the
// O(log) full-tile doubling passes of fs_mark (kept for A/B,
// ZKMI_FS_MARK=double).  Frame starts go to a per-tile uint16 list.
constexpr int64_t FS_LMAX = FS_S / 4;    // most frame starts a tile can hold

// One wave per tile: the wave stages the tile into its own 16 KiB of LDS
// with 16-byte loads, then lane 0 follows the chain there (an LDS hop is
// ~40 ns against ~250+ ns for an Infinity-Cache hit), 4 tiles per block.
constexpr int FS_WALK_TPB = 4;

__global__ __launch_bounds__(256) void fs_walk(const uint8_t* __restrict__ buf,
                                              int64_t n, int64_t maxp,
                                              int64_t tiles,
                                              const int64_t* __restrict__ ent,
                                              uint16_t* __restrict__ list,
                                              int64_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * FS_WALK_TPB + wv;
  if (t >= tiles) return;
  const int64_t e = ent[t];
  if (e == NONE) {
    if (lane == 0) counts[t] = 0;
    return;
  }
  uint8_t* sb = smem + wv * (FS_S + 16);
  const int64_t ts = t * FS_S;
  stage_tile<64>(buf, n, ts, sb, lane);
  // Wave-local staging (no workgroup barrier: sibling waves may have exited):
  // drain this wave's LDS writes before lane 0 reads them.
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const int32_t te = (int32_t)(min(ts + FS_S, n) - ts);   // tile-relative
  const int32_t nrel = (int32_t)min(n - ts, (int64_t)1 << 30);
  const int32_t maxp32 = (int32_t)min(maxp, (int64_t)1 << 30);
  // The walk is wave-UNIFORM: every lane runs it on scalar copies
  // (readfirstlane), so the loop is ~25 mostly-SALU instructions around one
  // LDS round trip per hop instead of a divergent lane-0 loop of ~45 VALU +
  // exec-mask instructions (measured ~500 cycles/hop).
  // The frame-start list is written IN PLACE over bytes already passed:
  // entry k lands at byte 2k while the walk is at >= 4k, so no byte still to
  // be read is overwritten, and no global store (with its vmcnt
  // back-pressure) sits inside the dependent-hop loop.
  uint16_t* Ls = (uint16_t*)sb;
  int32_t c = __builtin_amdgcn_readfirstlane((int32_t)(e - ts));
  int32_t cnt = 0;
  while (c < te) {
    const int32_t a = c & ~3;
    const uint32_t lo = *(const uint32_t*)(sb + a);
    const uint32_t hi = *(const uint32_t*)(sb + a + 4);
    const int32_t len = __builtin_amdgcn_readfirstlane(
        (int32_t)bswap32(__builtin_amdgcn_alignbyte(hi, lo, c & 3)));
    const int32_t nx = c + 4 + len;
    if ((c + 4 > nrel) | (len < 0) | (len > maxp32) | (nx > nrel)) break;
    if (lane == 0) Ls[cnt] = (uint16_t)c;
    ++cnt;
    c = nx;                                   // >= S ends the loop
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  uint16_t* L = list + t * FS_LMAX;
  for (int32_t k = lane; k < cnt; k += 64) L[k] = Ls[k];
  if (lane == 0) counts[t] = cnt;
}

// E' — list -> (body offset, length) table; one wave per tile, coalesced.
__global__ __launch_bounds__(256) void fs_write_list(
    const uint8_t* __restrict__ buf, int64_t tiles,
    const uint16_t* __restrict__ list, const int64_t* __restrict__ counts,
    const int64_t* __restrict__ base, int64_t* __restrict__ foff,
    int32_t* __restrict__ flen, int64_t cap, int64_t* __restrict__ result) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= tiles) return;
  const int lane = threadIdx.x & 63;
  const int64_t cnt = counts[t];
  const int64_t b = base[t];
  const int64_t ts = t * FS_S;
  const uint16_t* L = list + t * FS_LMAX;
  for (int64_t k = lane; k < cnt; k += 64) {
    const int64_t P = ts + L[k];
    const int64_t idx = b + k;
    if (idx < cap) {
      foff[idx] = P + 4;
      flen[idx] = ld_be32(buf + P);
    } else {
      result[3] = 1;
    }
  }
}

// ---- frontier pipeline, stages 2-4 -----------------------------------------
// Survivor slot s of tile t: surv[t*2+s] = (walker id << 16) | position, or
// -1; its frame starts R_s go to list[(t*2+s)*FS_LMAX ...], its count to
// rcount[t*2+s].

// Replace fe_pending(slot) in the tile's f0 row by the slot's final code.
ZK_DEV void fe_patch_row(uint16_t* row, int W, int lane,
                         const uint16_t fin[FE_NSURV]) {
  for (int j = lane; j < W / 8; j += 64) {
    uint4 v = ((const uint4*)row)[j];
    uint16_t* h = (uint16_t*)&v;
    bool any = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int sl = 0; sl < FE_NSURV; ++sl)
        if (h[k] == fe_pending(sl)) { h[k] = fin[sl]; any = true; }
    }
    if (any) ((uint4*)row)[j] = v;
  }
}

// A2 fs_survivor (LDS): one wave per tile; lane s walks survivor slot s of
// the staged tile (the two walks advance in lockstep, one LDS round trip per
// hop).  Frame starts go straight to global memory: those stores count in
// vmcnt, which the LDS hop loop never waits on.  16 KiB of LDS -> 9 tiles
// per CU: the variant for streams with few tiles (long chains per tile).
constexpr size_t FV_LDS = FS_S + 16;

__global__ __launch_bounds__(64) void fs_survivor(
    const uint8_t* __restrict__ buf, int64_t n, int64_t maxp, int32_t W,
    uint16_t* __restrict__ f0, const int32_t* __restrict__ surv,
    uint16_t* __restrict__ list, int32_t* __restrict__ rcount) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* sb = smem;                                      // [S + 16]
  const int lane = threadIdx.x;
  const int64_t t = blockIdx.x;
  const int64_t ts = t * FS_S;
  const int32_t sv = lane < FE_NSURV ? surv[t * FE_NSURV + lane] : -1;
  if (!__ballot(sv >= 0)) {                  // nothing pending in this tile
    if (lane < FE_NSURV) rcount[t * FE_NSURV + lane] = 0;
    return;
  }
  stage_tile<64>(buf, n, ts, sb, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const int32_t nrel = (int32_t)min(n - ts, (int64_t)1 << 30);
  const int32_t maxp32 = (int32_t)min(maxp, (int64_t)1 << 30);
  int32_t m = 0;
  uint16_t fin = 0;
  if constexpr (FE_NSURV == 1) {
    // one survivor: wave-uniform scalar walk.  The hot loop keeps only what
    // a clean hop needs (one unsigned length bound, one position bound that
    // folds "stays in the tile" and "fits the stream"); the hop that ends
    // the walk is re-classified exactly by fe_hop_len after the loop.  Frame
    // starts collect in a VGPR (entry k in lane k & 63, a v_cndmask, no exec
    // branching) and go out 64 at a time, IN PLACE over tile bytes already
    // passed (entry k at byte 2k while the walk is at >= 4k).
    int32_t c = __builtin_amdgcn_readfirstlane(sv) & 0xFFFF;
    uint16_t* Ls = (uint16_t*)sb;
    const int32_t lim = min(nrel + 1, (int32_t)FS_S);
    const uint32_t umax = (uint32_t)maxp32;
    uint32_t ent = 0;
    for (;;) {
      uint32_t lo, hi;
      fe_words(sb, c, lo, hi);
      const int32_t len = __builtin_amdgcn_readfirstlane(fe_len(lo, hi, c));
      const int32_t nx = c + 4 + len;
      if (((uint32_t)len > umax) | (nx >= lim)) break;
      ent = lane == (m & 63) ? (uint32_t)c : ent;
      ++m;
      if ((m & 63) == 0) Ls[m - 64 + lane] = (uint16_t)ent;
      c = nx;
    }
    {
      uint32_t lo, hi;
      fe_words(sb, c, lo, hi);
      const int32_t len = __builtin_amdgcn_readfirstlane(fe_len(lo, hi, c));
      int32_t q = 0;
      const uint16_t code = fe_hop_len(len, c, nrel, maxp32, q);
      if (!((code & F0_TERM) && code != F0_ESC)) {
        ent = lane == (m & 63) ? (uint32_t)c : ent;   // leaves the tile
        ++m;
        if ((m & 63) == 0) Ls[m - 64 + lane] = (uint16_t)ent;
      }
      fin = code;
    }
    if (lane < (m & 63)) Ls[(m & ~63) + lane] = (uint16_t)ent;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    uint16_t* L = list + t * FS_LMAX;
    for (int32_t k = lane; k < m; k += 64) L[k] = Ls[k];
    if (lane != 0) m = 0;                    // slot 0 lives in lane 0
  } else {
  bool a = sv >= 0;
  int32_t c = sv & 0xFFFF;
  uint16_t* L = list + (t * FE_NSURV + lane) * FS_LMAX;
  while (__ballot(a)) {
    if (a) {
      uint32_t lo, hi;
      fe_words(sb, c, lo, hi);
      int32_t q = 0;
      const uint16_t code = fe_hop(lo, hi, c, nrel, maxp32, q);
      if (code != FE_GO && (code & F0_TERM) && code != F0_ESC) {
        fin = code;                          // terminal: not a frame start
        a = false;
      } else {
        L[m++] = (uint16_t)c;
        if (code != FE_GO) { fin = code; a = false; }   // leaves the tile
        else c = q;
      }
    }
  }
  }
  if (lane < FE_NSURV) rcount[t * FE_NSURV + lane] = m;
  uint16_t fins[FE_NSURV];
#pragma unroll
  for (int sl = 0; sl < FE_NSURV; ++sl)
    fins[sl] = (uint16_t)__builtin_amdgcn_readlane((int)fin, sl);
  fe_patch_row(f0 + t * W, W, lane, fins);
}

// A2' fs_survivor_g: the same walks straight from global memory, no LDS.  A
// dependent hop costs more from L2 than from LDS (~0.4 vs ~0.1 us under
// load), but without the 16 KiB LDS tile a CU holds 32 walking waves instead
// of 9 and nothing is staged: the variant for streams with many tiles.
// Each slot is walked by a wave-uniform loop (two aligned dwords per hop +
// v_alignbyte); its frame starts collect in a VGPR (entry k in lane k & 63,
// one v_cndmask) and leave in one coalesced store per 64 hops.  4 tiles
// (waves) per block.
__global__ __launch_bounds__(256) void fs_survivor_g(
    const uint8_t* __restrict__ buf, int64_t n, int64_t maxp, int32_t W, int64_t tiles,
    uint16_t* __restrict__ f0, const int32_t* __restrict__ surv,
    uint16_t* __restrict__ list, int32_t* __restrict__ rcount) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= tiles) return;
  const int64_t ts = t * FS_S;
  const uint8_t* tb = buf + ts;
  const int32_t nrel = (int32_t)min(n - ts, (int64_t)1 << 30);
  const int32_t maxp32 = (int32_t)min(maxp, (int64_t)1 << 30);
  uint16_t fins[FE_NSURV];
  bool any_sv = false;
#pragma unroll
  for (int sl = 0; sl < FE_NSURV; ++sl) {
    const int32_t sv = __builtin_amdgcn_readfirstlane(
        surv[t * FE_NSURV + sl]);
    fins[sl] = 0;
    if (sv < 0) {
      if (lane == 0) rcount[t * FE_NSURV + sl] = 0;
      continue;
    }
    any_sv = true;
    uint16_t* L = list + (t * FE_NSURV + sl) * FS_LMAX;
    int32_t c = sv & 0xFFFF;
    int32_t m = 0;
    uint32_t ent = 0;
    uint16_t fin;
    // fast loop: one unsigned length bound and one position bound (stay in
    // the tile AND leave room for the next length word); the ending hop is
    // classified exactly afterwards
    const int32_t lim = min(nrel - 3, (int32_t)FS_S);
    const uint32_t umax = (uint32_t)maxp32;
    for (;;) {
      if (c >= lim) break;
      const int32_t a = c & ~3;
      const int32_t a2 = (a + 4 < nrel) ? a + 4 : a;
      const uint32_t w0 = *(const uint32_t*)(tb + a);
      const uint32_t w1 = *(const uint32_t*)(tb + a2);
      const int32_t len = __builtin_amdgcn_readfirstlane(fe_len(w0, w1, c));
      const int32_t nx = c + 4 + len;
      if (((uint32_t)len > umax) | (nx > nrel) | (nx >= (int32_t)FS_S)) break;
      ent = lane == (m & 63) ? (uint32_t)c : ent;   // entry m -> lane m&63
      ++m;
      if ((m & 63) == 0) L[m - 64 + lane] = (uint16_t)ent;
      c = nx;
    }
    if (c + 4 > nrel) {
      fin = (uint16_t)(F0_TERM | c);
    } else {
      const int32_t a = c & ~3;
      const int32_t a2 = (a + 4 < nrel) ? a + 4 : a;
      const uint32_t w0 = *(const uint32_t*)(tb + a);
      const uint32_t w1 = *(const uint32_t*)(tb + a2);
      const int32_t len = __builtin_amdgcn_readfirstlane(fe_len(w0, w1, c));
      int32_t q = 0;
      fin = fe_hop_len(len, c, nrel, maxp32, q);
      if (!((fin & F0_TERM) && fin != F0_ESC)) {   // leaves: a frame start
        ent = lane == (m & 63) ? (uint32_t)c : ent;
        ++m;
        if ((m & 63) == 0) L[m - 64 + lane] = (uint16_t)ent;
      }
    }
    if (lane < (m & 63)) L[(m & ~63) + lane] = (uint16_t)ent;
    if (lane == 0) rcount[t * FE_NSURV + sl] = m;
    fins[sl] = fin;
  }
  if (any_sv) fe_patch_row(f0 + t * W, W, lane, fins);
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

__global__ __launch_bounds__(64) void fs_survivor_r(
    const uint8_t* __restrict__ buf, int64_t n, int64_t maxp, int32_t W,
    uint16_t* __restrict__ f0, const int32_t* __restrict__ surv,
    uint16_t* __restrict__ list, int32_t* __restrict__ rcount) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[FR_RING];
  const int lane = threadIdx.x;
  const int64_t t = blockIdx.x;
  const int64_t ts = t * FS_S;
  // one survivor per tile (FE_NSURV == 1; the launcher checks)
  const int32_t sv = __builtin_amdgcn_readfirstlane(surv[t * FE_NSURV]);
  if (sv < 0) {
    if (lane == 0) rcount[t * FE_NSURV] = 0;
    return;
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
    }
  }
  if (lane < (m & 63)) L[(m & ~63) + lane] = (uint16_t)ent;
  if (lane == 0) rcount[t * FE_NSURV] = m;
  uint16_t fins[FE_NSURV] = {fin};
  fe_patch_row(f0 + t * W, W, lane, fins);
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

struct FsPlan {
  int levels;
  int64_t units[FS_MAXL];
  int64_t usize[FS_MAXL];
  size_t off_f0, off_fl[FS_MAXL], off_ent[FS_MAXL], off_bits, off_cnt,
      off_base, off_scan, off_list, off_pre, off_surv, off_rcnt, off_npre,
      total;
};

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
  for (int l = 1; l < p.levels; ++l)
    p.off_fl[l] = take((size_t)p.units[l] * W * 8);
  for (int l = 0; l < p.levels; ++l) p.off_ent[l] = take((size_t)p.units[l] * 8);
  p.off_bits = take((size_t)tiles * (FS_S / 32) * 4);
  p.off_cnt = take((size_t)tiles * 8);
  p.off_base = take((size_t)tiles * 8);
  p.off_scan = take((size_t)zk_scan_workspace(tiles) * 8);
  p.off_list = take((size_t)tiles * FE_NSURV * FS_LMAX * 2);
  p.off_pre = take((size_t)tiles * FS_LMAX * 2);
  p.off_surv = take((size_t)tiles * FE_NSURV * 4);
  p.off_rcnt = take((size_t)tiles * FE_NSURV * 4);
  p.off_npre = take((size_t)tiles * 4);
  p.total = o;
  return p;
}

}  // namespace zk

extern "C" {

// Sized for the largest window (FS_W), an upper bound for any window.
int64_t zk_frame_scan_workspace(int64_t n) {
  return (int64_t)zk::fs_plan(n, zk::FS_W).total;
}

// result (device int64[4]): [0] frames written, [1] stop offset (consumed
// bytes; start of the carry or of the bad frame), [2] 1 if the stop is a
// BAD_LENGTH frame, [3] 1 if the frame table overflowed `cap`.
//
// `window` (256 / 512 / 1024 / 2048 bytes) is the fast-path entry window per
// 16 KiB tile: a chain can only enter a tile inside it when frames are <=
// window bytes, so the frontier walks `window` speculative entry points per
// tile and the composition tables hold `window` entries per unit.  Frames
// longer than the window stay exact (walked in global memory for the tiles
// they land in), so the window is a performance hint: the smallest one
// covering the stream's usual frame size makes the scan cheapest.
int zk_frame_scan2(const uint8_t* buf, int64_t n, int64_t maxp, uint8_t* ws,
                   int64_t ws_bytes, int64_t* foff, int32_t* flen, int64_t cap,
                   int64_t* result, int32_t window, hipStream_t st) {
  using namespace zk;
  const int W = window <= 256 ? 256 : window <= 512 ? 512
              : window <= 1024 ? 1024 : (int)FS_W;
  FsPlan p = fs_plan(n, W);
  if ((int64_t)p.total > ws_bytes) return -1;
  hipMemsetAsync(result, 0, 4 * sizeof(int64_t), st);
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
  // ZKMI_FS_SCAN: "frontier" (default) | "jump" (fs_exits + fs_walk) |
  // "double" (fs_exits + fs_mark doubling) — the older paths stay for A/B.
  static int mode = -1;
  if (mode < 0) {
    const char* m = getenv("ZKMI_FS_SCAN");
    mode = !m ? 0 : (m[0] == 'j' ? 1 : (m[0] == 'd' ? 2 : 0));
  }
  if (mode != 0 && W != FS_W) return -2;       // A/B paths: full window only
  uint16_t* f0w = (uint16_t*)(ws + p.off_f0);
  uint32_t* bits = (uint32_t*)(ws + p.off_bits);
  int64_t* cnt = (int64_t*)(ws + p.off_cnt);
  int64_t* base = (int64_t*)(ws + p.off_base);
  uint16_t* list = (uint16_t*)(ws + p.off_list);
  uint16_t* pre = (uint16_t*)(ws + p.off_pre);
  int32_t* surv = (int32_t*)(ws + p.off_surv);
  int32_t* rcnt = (int32_t*)(ws + p.off_rcnt);
  int32_t* npre = (int32_t*)(ws + p.off_npre);
  if (mode == 0) {
    switch (W) {
      case 256:
        fs_frontier<256><<<(unsigned)tiles, FE_T, fe_lds(256), st>>>(
            buf, n, maxp, f0w, surv);
        break;
      case 512:
        fs_frontier<512><<<(unsigned)tiles, FE_T, fe_lds(512), st>>>(
            buf, n, maxp, f0w, surv);
        break;
      case 1024:
        fs_frontier<1024><<<(unsigned)tiles, FE_T, fe_lds(1024), st>>>(
            buf, n, maxp, f0w, surv);
        break;
      default:
        fs_frontier<(int)FS_W><<<(unsigned)tiles, FE_T, fe_lds((int)FS_W),
                                 st>>>(buf, n, maxp, f0w, surv);
    }
    ZK_LAUNCH_CHECK();
    // Survivor walk: through a 4 KiB LDS ring (default; LDS hop latency at
    // up to 32 walks per CU).  ZKMI_FS_SURVIVOR=lds|global|ring selects the
    // whole-tile LDS walk (9 walks per CU) or the L2 walk for A/B runs.
    static int sv_force = -1;
    if (sv_force < 0) {
      const char* m = getenv("ZKMI_FS_SURVIVOR");
      sv_force = !m ? 0 : (m[0] == 'l' ? 1 : (m[0] == 'g' ? 2
                                               : (m[0] == 'r' ? 3 : 0)));
    }
    const int sv_mode = sv_force ? sv_force : 3;
    if (sv_mode == 3 && FE_NSURV == 1)
      fs_survivor_r<<<(unsigned)tiles, 64, 0, st>>>(buf, n, maxp, W, f0w,
                                                   surv, list, rcnt);
    else if (sv_mode == 1)
      fs_survivor<<<(unsigned)tiles, 64, FV_LDS, st>>>(buf, n, maxp, W, f0w,
                                                      surv, list, rcnt);
    else
      fs_survivor_g<<<(unsigned)((tiles + 3) / 4), 256, 0, st>>>(
          buf, n, maxp, W, tiles, f0w, surv, list, rcnt);
  } else {
    const size_t lds_a = FS_S * 2 + FS_LIST * 2 + (FS_T / 64 + 1) * 8;
    fs_exits<<<(unsigned)tiles, FS_T, lds_a, st>>>(buf, n, maxp, f0w);
  }
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
  if (mode == 0) {
    fs_join<<<wblocks, 256, 0, st>>>(buf, n, maxp, tiles, c.ent[0], list,
                                     rcnt, pre, npre, cnt);
  } else if (mode == 2) {
    fs_mark<<<(unsigned)tiles, FS_T, FS_S * 5, st>>>(buf, n, maxp, c.ent[0],
                                                    bits, cnt);
  } else {
    fs_walk<<<(unsigned)((tiles + FS_WALK_TPB - 1) / FS_WALK_TPB), 256,
              FS_WALK_TPB * (FS_S + 16), st>>>(buf, n, maxp, tiles, c.ent[0],
                                               list, cnt);
  }
  ZK_LAUNCH_CHECK();
  int rc = zk_scan_excl_i64(cnt, base, tiles, result + 0,
                            (int64_t*)(ws + p.off_scan), st);
  if (rc) return rc;
  if (mode == 0) {
    fs_write_join<<<wblocks, 256, 0, st>>>(buf, tiles, pre, npre, list, cnt,
                                           base, foff, flen, cap, result);
  } else if (mode == 2) {
    fs_write<<<(unsigned)tiles, 256, 0, st>>>(buf, bits, base, foff, flen,
                                             cap, result);
  } else {
    fs_write_list<<<wblocks, 256, 0, st>>>(buf, tiles, list, cnt, base, foff,
                                           flen, cap, result);
  }
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_frame_scan(const uint8_t* buf, int64_t n, int64_t maxp, uint8_t* ws,
                  int64_t ws_bytes, int64_t* foff, int32_t* flen, int64_t cap,
                  int64_t* result, hipStream_t st) {
  return zk_frame_scan2(buf, n, maxp, ws, ws_bytes, foff, flen, cap, result,
                        (int32_t)zk::FS_W, st);
}

}  // extern "C"

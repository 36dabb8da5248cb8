// K1 — parallel length-prefixed frame scan.
//
// Reference: ZKDecodeStream._transform (lib/zk-streams.js:39-65) walks the
// i32-BE length chain one frame at a time and memmoves the remainder per
// packet (O(bytes x packets)).  The chain is inherently
// sequential; we make it parallel without speculation errors, over 4 KiB
// tiles, in four launches:
//
//  fs_tile   ONE WAVE per tile (4 per workgroup, independent, no barriers).
//            The tile is staged into the wave's LDS once; everything else
//            runs there:
//            1. merging frontier: one walker per window entry e < W (the
//               only places a chain can enter a tile when frames are <= W
//               bytes); each round every live walker hops and claims the
//               position it lands on in an owner table; a walker landing on
//               a claimed position has the same future as the claimant and
//               stops.  Garbage entries die on their first hop (random
//               bytes read as a length are huge or negative), the true
//               chain's entries merge within a hop, so after a few rounds
//               one walker — the survivor — is left;
//            2. the survivor walks to the tile end, recording its frame
//               starts (LDS, one hop = one LDS round trip);
//            3. every exit a walker took into the next tile's window is a
//               candidate entry of that tile; the preferred one (the
//               survivor's exit) and up to four others go out in ONE packed
//               64-bit word (ready bit + five 12-bit offsets, a relaxed
//               agent-scope store: no release fence, which costs an L2
//               writeback per wave on a multi-XCD part).  The true chain's
//               exit is among the in-window exits when frames are <= W.
//               The tile takes the word of the tile before (a one-step wait:
//               that wave started earlier and does the same work) and walks
//               each candidate in LDS: a garbage chain of the tile before,
//               read on here, dies on a bad length within a few hops; the
//               first candidate whose chain survives the tile is the entry.
//               (Round 2 first published only the last surviving walker's
//               exit: on structured replies of a few hundred bytes a slow
//               garbage crawler outlived the true chain in ~20 % of the
//               tiles, and every such tile cost a serial repair.)
//            4. from the entry, a short walk (usually 1-5 frames) until the
//               chain meets the survivor's recorded path (merge-walk against
//               the sorted list), the tile end or a terminal.
//            The entry is exact unless a frame longer than the window ends
//            in the tile before or two candidates' chains both survive.
//  fs_check  one thread per tile (a grid): is tile k's entry tile k-1's
//            exit, is the tile terminal; frame counts scanned per block of
//            256 tiles.  The leftmost broken link / terminal go to fs_link
//            as one atomic per block.
//  fs_link   No broken link before the first terminal (the usual case):
//            one workgroup scans the block totals, done.  A few broken
//            links (<= 64): chased — from each, forward while the next link
//            stays broken, the exact entry of a tile looked up among the
//            candidates fs_tile walked (their exits are its entry -> exit
//            map), so a run of tiles costs a few instructions each; the
//            looked-up tiles are then re-walked in parallel over the grid
//            of 64 workgroups for their frame lists.  Many broken links: a
//            fix-point in grid rounds (every broken link re-walked in
//            parallel from the exit before it).  Whatever neither settles
//            is finished serially, tiles covered whole by one frame filled
//            in one step; then the counts are scanned up to the first
//            terminal: row bases and result[0..3].
//  fs_rows   one wave per tile writes its (body offset, length) rows.
//
// The stream length is read ON THE DEVICE (n = min(*n_dev, n_cap), e.g. an
// encoder's total): the grids cover the buffer capacity, tiles past the
// length return at once, and no byte past it is read.  BAD_LENGTH is
// reported at the exact frame (result[1] = its offset, result[2] = 1), the
// consumed prefix ends at the last complete frame, and a partial trailing
// frame is left for the next call (carry), like the reference's buffer.
//
// History (profiles/): round 1 scanned 16 KiB tiles with a 256-thread
// frontier block, a separate survivor kernel through a 4 KiB LDS ring, and
// log-depth function composition + push-down + join + count scan + write
// (13-15 launches, ~130 us per 200 MB reply stream on the composition
// alone).  A single-pass decoupled look-back replacing the composition
// stalled: with every tile resident at once, each tile looked back across
// all the tiles before it (~100 us).  The survivor's 2 KiB ring reloads
// stalled on HBM latency at every chunk (~1 us per reply frame).  Staging
// a 4 KiB tile once per wave removes both.
#include "zk_common.h"

namespace zk {

constexpr int FT_S = 4096;                 // tile bytes
constexpr int FT_LMAX = FT_S / 4;          // most frame starts a tile holds
constexpr int FT_STAGE = FT_S + 16;        // staged bytes (+ length overhang)
constexpr int64_t TERM = (int64_t)1 << 62;
constexpr int64_t TBAD = (int64_t)1 << 60;
constexpr int64_t FC_MAXP = (int64_t)1 << 24;
constexpr int FC_WIN = 4096;               // fs_link's staged walk window
constexpr int FC_TAILWIN = 8192;           // the serial tail's (one wave)
// fs_link threads (512: 256 VGPRs a lane — with 1024 the chase and the walk
// inlined together spilled to scratch, 0.64 us a looked-up tile)
constexpr int FL_T = 512;
constexpr int FL_U = 8;                    // fs_link loads per batch
// Bound of fs_tile's wait for the tile before (100 MHz ticks, 2 ms): normal
// waits are tens of microseconds; past the bound the tile takes no
// speculated entry and fs_link re-walks it from the exact one.
constexpr uint64_t FT_WAIT_TICKS = 200000;

// The scanned length: a producer's device-side byte count clamped to the
// buffer capacity (null: the capacity itself, a host-known length).
ZK_DEV int64_t stream_len(const int64_t* n_dev, int64_t n_cap) {
  if (n_dev == nullptr) return n_cap;
  const int64_t v = *n_dev;
  return v < 0 ? 0 : (v < n_cap ? v : n_cap);
}

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

// Chain statistics after the X flags: [0] tiles fs_link's chases looked up,
// [1] tiles without a speculated entry, [2] tiles re-walked by fs_link, [3]
// fs_link repair rounds (zk_frame_scan_stats reads them).
ZK_DEV void fc_stat(uint64_t* stats, int k, uint32_t v) {
  __hip_atomic_fetch_add((uint32_t*)&stats[k], v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}

// Big-endian i32 at byte p of an LDS image (two aligned dwords + alignbyte).
ZK_DEV int32_t lds_be32(const uint8_t* sb, int32_t p) {
  const int32_t a = p & ~3;
  const uint32_t lo = *(const uint32_t*)(sb + a);
  const uint32_t hi = *(const uint32_t*)(sb + a + 4);
  return (int32_t)bswap32(__builtin_amdgcn_alignbyte(hi, lo, p & 3));
}

// ---- LDS layout of fs_tile<W> (5.4 KiB per wave) ----------------------------
// tile [FT_STAGE] | claimed bits [FT_S/32] | survivor bits [FT_S/32] |
// compaction scratch [64] (uint16) | exit candidate bits [FT_XW]
constexpr int FT_BITS = FT_S / 32;         // uint32 words per position map
constexpr int FT_XW = 2048 / 32;           // exit candidates: the next tile's
                                           // window positions (W <= 2048)
constexpr int FT_LDS = FT_STAGE + 2 * FT_BITS * 4 + 64 * 2 + FT_XW * 4;

// One hop from tile-relative p (< FT_S).  Returns 0 and q (in-tile
// successor), 1 for a terminal (the chain ends in the tile), or 2 and the
// exit x (tile end + x) when the frame leaves the tile.
// `minb`: the frontier's plausibility floor on a frame body (the smallest
// ZooKeeper body is 8 bytes: a ping's xid + type).  Speculative walkers
// reading a shorter length die at once instead of crawling 4 bytes a hop
// through zero header fields; exactness is untouched (a real frame that
// short only costs its tile the speculated entry, fs_link repairs it).
ZK_DEV int ft_hop(const uint8_t* sb, int32_t p, int32_t nrel, int32_t maxp,
                  int32_t minb, int32_t& q) {
  if (p >= nrel) return 1;                 // the stream ended before p
  const int32_t len = lds_be32(sb, p);
  const int32_t nx = p + 4 + len;
  if ((p + 4 > nrel) | (len < minb) | (len > maxp) | (nx > nrel)) return 1;
  q = nx;
  return nx >= FT_S ? 2 : 0;
}

// Claim position q in a bit map: true when this lane is the first (the
// fetch-or's old bit was clear).  Lanes of one instruction hitting the same
// word are serialised by the LDS unit, so exactly one of them wins.
ZK_DEV bool ft_claim(uint32_t* bits, int32_t q) {
  const uint32_t b = 1u << (q & 31);
  return (__hip_atomic_fetch_or(&bits[q >> 5], b, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_WAVEFRONT) & b) == 0;
}

// per-tile record: meta = cnt | np << 11 | (js + 1) << 22 | term << 33 |
// bad << 34; entry = the entry used (-1: none, the tile before had no
// speculated exit); exit = exit position or the terminal's position.
struct FcWalk {
  int64_t exit;
  int32_t cnt;       // frame starts of the tile on the chain
  int32_t np;        // of which walked before meeting the survivor (pre[])
  int32_t js;        // survivor list index the rest starts at (-1: none)
  bool term, bad;
};
ZK_DEV int64_t fc_meta(const FcWalk& w) {
  return (int64_t)w.cnt | ((int64_t)w.np << 11) | ((int64_t)(w.js + 1) << 22) |
         ((int64_t)w.term << 33) | ((int64_t)w.bad << 34);
}
ZK_DEV int32_t m_cnt(int64_t m) { return (int32_t)(m & 0x7FF); }
ZK_DEV int32_t m_np(int64_t m) { return (int32_t)((m >> 11) & 0x7FF); }
ZK_DEV int32_t m_js(int64_t m) { return (int32_t)((m >> 22) & 0x7FF) - 1; }
ZK_DEV bool m_term(int64_t m) { return (m >> 33) & 1; }
ZK_DEV bool m_bad(int64_t m) { return (m >> 34) & 1; }
// a tile whose exact entry, exit and frame count fs_link's chase looked up:
// its recorded frame starts are still the old entry's, so fs_rows walks it
constexpr int64_t M_STALE = (int64_t)1 << 35;
ZK_DEV bool m_stale(int64_t m) { return (m >> 35) & 1; }

// Resolve the survivor's end code `send` into the walk result's exit.
ZK_DEV void fc_join_end(FcWalk& r, int64_t send, int64_t n) {
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

// Membership of crel in the sorted survivor list L[0..m0) (merge-walk: the
// walk only moves forward, so the 64-entry window lv only moves forward).
// Returns the list index or -1.
template <typename LoadL>
ZK_DEV int32_t fc_member(uint32_t crel, int32_t m0, int32_t& lb, uint32_t& lv,
                         int lane, LoadL loadL) {
  while (lb + 64 < m0 &&
         crel > (uint32_t)__builtin_amdgcn_readlane((int)lv, 63)) {
    lb += 64;
    lv = lb + lane < m0 ? loadL(lb + lane) : 0xFFFFFFFFu;
  }
  const uint64_t hit = __ballot(lv == crel);
  return hit ? lb + (int32_t)__builtin_ctzll(hit) : -1;
}

// Record frame start c as entry m of a list in global memory: lane m & 63
// keeps it in `ent`, every 64 entries leave in one coalesced store.
ZK_DEV void ft_record(uint16_t* L, int32_t& m, uint32_t& ent, int32_t c,
                      int lane) {
  ent = lane == (m & 63) ? (uint32_t)c : ent;
  ++m;
  if ((m & 63) == 0) L[m - 64 + lane] = (uint16_t)ent;
}

// Mark a walker's exit x (offset into the next tile) as an entry candidate
// of that tile; exits past the window cannot be the chain's (frames <= W).
ZK_DEV bool ft_mark_exit(uint32_t* xbits, int32_t x, int W) {
  if (x < 0 || x >= W) return false;
  __hip_atomic_fetch_or(&xbits[x >> 5], 1u << (x & 31), __ATOMIC_RELAXED,
                        __HIP_MEMORY_SCOPE_WAVEFRONT);
  return true;
}

// The chain from tile-relative candidate entry e, walked in LDS (wave-
// uniform): does it survive this tile, and where does it leave it?
// Returns the absolute exit (>= the tile end) when it leaves the tile, or
// meets the survivor's path and the survivor leaves (its exit `send`),
// packed with the number of frames the chain starts in this tile
// (cx_exit / cx_cnt); FC_DEAD when it hits a bad length or meets a
// survivor that ends on one; FC_LIVE when it survives without a known exit
// (it reaches the stream end, or meets a survivor that ends there).
// fs_link's chase takes these as the tile's entry -> (exit, count) map.
constexpr int64_t FC_DEAD = -1;
constexpr int64_t FC_LIVE = -2;
constexpr int CX_SHIFT = 48;
ZK_DEV int64_t cx_exit(int64_t v) {
  return v < 0 ? v : v & (((int64_t)1 << CX_SHIFT) - 1);
}
ZK_DEV int32_t cx_cnt(int64_t v) { return v < 0 ? 0 : (int32_t)(v >> CX_SHIFT); }

ZK_DEV int64_t ft_cand(const uint8_t* sb, const uint32_t* sbits, int32_t e,
                       int32_t nrel, int32_t maxp, int64_t send, int64_t n,
                       int64_t ts, int32_t m, int lane) {
  int32_t c = e;
  int32_t hops = 0;
  for (;;) {
    if (c >= FT_S) return (ts + c) | ((int64_t)hops << CX_SHIFT);
    if (ts + c >= n) return FC_LIVE;
    // the survivor-map word and the length word, read together (the map
    // is all zero without a survivor)
    const uint32_t smw = sbits[c >> 5];
    const int32_t lraw = lds_be32(sb, c);
    if ((smw >> (c & 31)) & 1u) {
      if (send & TERM) return (send & TBAD) ? FC_DEAD : FC_LIVE;
      // joined: the survivor's frames from its start at c on (their index
      // is the number of survivor starts below c; two map words a lane)
      const int32_t cw = c >> 5;
      int32_t below = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int32_t wi = lane + 64 * h;
        const uint32_t wd = sbits[wi];
        below += wi < cw ? __popc(wd)
                         : (wi == cw ? __popc(wd & ((1u << (c & 31)) - 1u))
                                     : 0);
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) below += __shfl_xor(below, d, 64);
      return send | ((int64_t)(hops + m - below) << CX_SHIFT);
    }
    if (c + 4 > nrel) return FC_LIVE;
    const int32_t len = __builtin_amdgcn_readfirstlane(lraw);
    if ((uint32_t)len > (uint32_t)maxp) return FC_DEAD;
    const int32_t nx = c + 4 + len;
    if (nx > nrel) return FC_LIVE;
    ++hops;
    c = nx;
  }
}

// Frontier passes past the window (fs_tile<W, true>, streams whose frames
// may be longer than the window): when a frame longer than the window
// covers [0, W) of a tile, every walker starts inside its body and dies
// (body bytes read as lengths are implausible), so no survivor is left.
// The frontier then runs again from [base, base + W) for base = W, 2W, ...
// until a walker survives: the chain resumes after that frame.  Positions
// the dead walkers claimed keep their meaning (a chain through one dies
// too).  Kept out of the usual path (its own function, only instantiated
// for LONG): a loop around the main frontier cost the GET step 9 %.
template <int W>
ZK_DEV void ft_frontier_passes(const uint8_t* sb, uint32_t* claimed,
                               uint32_t* xbits, uint16_t* scratch,
                               int32_t nrel, int32_t maxp32, int32_t minb,
                               int lane, uint32_t& lastx, int& round,
                               int32_t& mp, bool& ma) {
  constexpr int K = W / 64;
  for (int32_t base = W; base < FT_S && base < nrel && __ballot(ma) == 0;
       base += W) {
    for (int k = lane; k < W / 32; k += 64)
      claimed[base / 32 + k] = 0xFFFFFFFFu;
    __builtin_amdgcn_wave_barrier();
    int32_t p[K];
    uint32_t act = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      p[k] = base + lane + 64 * k;
      act |= 1u << k;
    }
    int32_t live = W;
    while (live > 64) {
      int32_t q[K];
      int code[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        q[k] = 0;
        code[k] = (act >> k) & 1 ? ft_hop(sb, p[k], nrel, maxp32, minb, q[k])
                                 : 1;
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (!((act >> k) & 1)) continue;
        if (code[k] == 0 && ft_claim(claimed, q[k])) {
          p[k] = q[k];
        } else {
          if (code[k] == 2 && ft_mark_exit(xbits, q[k] - FT_S, W))
            lastx = max(lastx, ((uint32_t)round << 16) |
                                   (uint32_t)(q[k] - FT_S));
          act &= ~(1u << k);
        }
      }
      ++round;
      int c = __popc(act);
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
      live = c;
    }
    {
      const uint32_t mine = __popc(act);
      uint32_t incl = mine;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      uint32_t o = incl - mine;
#pragma unroll
      for (int k = 0; k < K; ++k)
        if ((act >> k) & 1) scratch[o++] = (uint16_t)p[k];
      __builtin_amdgcn_wave_barrier();
      ma = lane < live;
      mp = ma ? (int32_t)scratch[lane] : 0;
      __builtin_amdgcn_wave_barrier();
    }
    while (live > 1) {
      int32_t q = 0;
      const int code = ma ? ft_hop(sb, mp, nrel, maxp32, minb, q) : 1;
      if (ma) {
        if (code == 0 && ft_claim(claimed, q)) {
          mp = q;
        } else {
          if (code == 2 && ft_mark_exit(xbits, q - FT_S, W))
            lastx = max(lastx, ((uint32_t)round << 16) | (uint32_t)(q - FT_S));
          ma = false;
        }
      }
      ++round;
      live = __popcll(__ballot(ma));
    }
  }
}

template <int W, bool LONG>
__global__ __launch_bounds__(256) void fs_tile(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ n_dev,
    int64_t n_cap, int64_t maxp, uint16_t* __restrict__ list,
    uint16_t* __restrict__ pre, int64_t* __restrict__ sx, uint64_t* lbw,
    int64_t* __restrict__ rec_entry, int64_t* __restrict__ rec_exit,
    int64_t* __restrict__ rec_meta, int32_t* __restrict__ rcount,
    int64_t ntiles_cap, int64_t* __restrict__ dbg, int32_t minb,
    int32_t tflags, int64_t* __restrict__ cx) {
  const bool nospec = tflags & 1;
  const int32_t misspec = tflags >> 8;
  constexpr int K = W / 64;                 // window entries per lane
  constexpr int XW = W / 32;                // candidate words used
  static_assert(W % 64 == 0 && K >= 1 && K <= 32, "window");
  // one tile per wave; a block's waves work independently (no barriers),
  // each in its own LDS slice
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_all[];
  uint8_t* smem = smem_all +
                  __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) *
                      FT_LDS;
  uint8_t* sb = smem;
  uint32_t* claimed = (uint32_t*)(smem + FT_STAGE);
  uint32_t* sbits = claimed + FT_BITS;       // survivor frame starts
  uint16_t* scratch = (uint16_t*)(sbits + FT_BITS);
  uint32_t* xbits = (uint32_t*)(scratch + 64);    // exits into the next tile
  const int lane = threadIdx.x & 63;
  const int64_t n = stream_len(n_dev, n_cap);
  const int64_t ntiles = (n + FT_S - 1) / FT_S;
  uint64_t* stats = &lbw[2 * ntiles_cap];
  // Tiles in workgroup order.  (An atomic ticket counter serialised every
  // wave's start at ~12 ns per ticket — one device-scope atomic address —
  // and paced the whole scan.)  The wait for the tile before (step 3) is
  // bounded, so no dispatch order can deadlock it.
  // (readfirstlane: the wave index is wave-uniform, and saying so keeps
  // the tile's positions and the walks' control in SGPRs)
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (t >= ntiles) return;
  const int64_t t_0 = dbg ? wall_clock64() : 0;
  const int64_t ts = t * FT_S;
  const int64_t tend = ts + FT_S;
  const int32_t nrel = (int32_t)min(n - ts, (int64_t)1 << 30);
  const int32_t maxp32 = (int32_t)maxp;

  // ---- stage the tile (all loads issued before the first LDS write) ------
  {
    constexpr int PER = FT_S / 16 / 64;     // 4 x 16 B per lane
    uint4 v[PER];
    uint4 pad = make_uint4(0, 0, 0, 0);
    if (ts + FT_STAGE <= n) {
#pragma unroll
      for (int j = 0; j < PER; ++j)
        __builtin_memcpy(&v[j], buf + ts + 16 * (lane + 64 * j), 16);
      if (lane == 0) __builtin_memcpy(&pad, buf + ts + FT_S, 16);
    } else {
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        uint8_t* b = (uint8_t*)&v[j];
        const int64_t g = ts + 16 * (lane + 64 * j);
        for (int k = 0; k < 16; ++k) b[k] = g + k < n ? buf[g + k] : 0;
      }
      if (lane == 0) {
        uint8_t* b = (uint8_t*)&pad;
        for (int k = 0; k < 16; ++k) b[k] = tend + k < n ? buf[tend + k] : 0;
      }
    }
    // window positions start claimed (each by its own walker)
    for (int k = lane; k < 2 * FT_BITS; k += 64)
      claimed[k] = k < W / 32 ? 0xFFFFFFFFu : 0u;
    if (lane < FT_XW) xbits[lane] = 0u;
#pragma unroll
    for (int j = 0; j < PER; ++j) *(uint4*)(sb + 16 * (lane + 64 * j)) = v[j];
    if (lane == 0) *(uint4*)(sb + FT_S) = pad;
  }
  const int64_t t_s = dbg ? (__builtin_amdgcn_s_waitcnt(0), wall_clock64()) : 0;
  // ---- 1. merging frontier ------------------------------------------------
  // Dense rounds: lane holds walkers e = lane + 64k.  A walker hops, then
  // claims its landing position with one fetch-or; landing on a claimed
  // position means merging into that chain, so it stops.  A round is two
  // LDS round trips (length words, claim) for all K walkers at once.
  // Every walker that leaves the tile marks its exit in `xbits` when it
  // lands inside the next tile's window: the candidate entries of the
  // next tile.  With frames <= W the true chain's exit is always one of
  // them (whichever walker carries the true chain leaves the tile there).
  int32_t p[K];
  uint32_t act = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    p[k] = lane + 64 * k;
    act |= 1u << k;
  }
  // `lastx` = (round << 16 | x) of the latest in-window exit the frontier
  // took: the preferred candidate when the survivor does not leave
  uint32_t lastx = 0;
  int round = 1;
  int32_t live = W;
  while (live > 64) {
    int32_t q[K];
    int code[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      q[k] = 0;
      code[k] = (act >> k) & 1 ? ft_hop(sb, p[k], nrel, maxp32, minb, q[k]) : 1;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (!((act >> k) & 1)) continue;
      if (code[k] == 0 && ft_claim(claimed, q[k])) {
        p[k] = q[k];
      } else {
        if (code[k] == 2 && ft_mark_exit(xbits, q[k] - FT_S, W))
          lastx = max(lastx, ((uint32_t)round << 16) | (uint32_t)(q[k] - FT_S));
        act &= ~(1u << k);
      }
    }
    ++round;
    int c = __popc(act);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
    live = c;
  }
  // sparse rounds: one walker per lane
  int32_t mp;
  bool ma;
  {
    uint32_t cnt_before = 0;
    {
      const uint32_t mine = __popc(act);
      uint32_t incl = mine;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      cnt_before = incl - mine;
    }
    uint32_t o = cnt_before;
#pragma unroll
    for (int k = 0; k < K; ++k)
      if ((act >> k) & 1) scratch[o++] = (uint16_t)p[k];
    __builtin_amdgcn_wave_barrier();
    ma = lane < live;
    mp = ma ? (int32_t)scratch[lane] : 0;
  }
  while (live > 1) {
    int32_t q = 0;
    const int code = ma ? ft_hop(sb, mp, nrel, maxp32, minb, q) : 1;
    if (ma) {
      if (code == 0 && ft_claim(claimed, q)) {
        mp = q;
      } else {
        if (code == 2 && ft_mark_exit(xbits, q - FT_S, W))
          lastx = max(lastx, ((uint32_t)round << 16) | (uint32_t)(q - FT_S));
        ma = false;
      }
    }
    ++round;
    live = __popcll(__ballot(ma));
  }
  if constexpr (LONG) {
    ft_frontier_passes<W>(sb, claimed, xbits, scratch, nrel, maxp32, minb,
                          lane, lastx, round, mp, ma);
  }
  const int64_t t_f = dbg ? wall_clock64() : 0;
  // ---- 2. the survivor walks to the tile end ------------------------------
  int64_t send = -1;
  int32_t m = 0;
  uint16_t* L = list + t * FT_LMAX;
  const uint64_t sm = __ballot(ma);
  if (sm) {
    const int sl = (int)__builtin_ctzll(sm);
    int32_t c = __builtin_amdgcn_readlane(mp, sl);
    uint32_t ent = 0;
    // The hot loop of the scan (one hop per frame of the tile, serial):
    // kept to a few scalar compares per hop — one unsigned test covers a
    // negative or oversize length, one bound (min(tile end, stream end))
    // both ways out, and the frame start goes into lane m & 63 of `ent`
    // (a compare and a select).  The rare exits are classified on the way
    // out.
    // (The round-2 loop spent ~45 instructions per hop on mixed VALU/SALU
    // tests; at ~7 waves per SIMD that issue cost, not the LDS latency,
    // set the ~300 ns per hop measured with ZKMI_FS_DBG.)
    const int32_t lim = min((int32_t)FT_S, nrel);
    if (c >= nrel) {
      send = TERM | (ts + c);                // reached the stream end
    } else {
      int32_t len, nx;
      bool ok;
      for (;;) {
        len = __builtin_amdgcn_readfirstlane(lds_be32(sb, c));
        nx = c + 4 + len;
        ok = (uint32_t)len <= (uint32_t)maxp32 && nx <= nrel;
        if (!ok) break;                      // one exit test per hop
        ent = lane == (m & 63) ? (uint32_t)c : ent;
        ++m;
        if ((m & 63) == 0) L[m - 64 + lane] = (uint16_t)ent;
        if (nx >= lim) break;
        c = nx;
      }
      if (!ok) {
        const bool bad = (c + 4 <= nrel) && ((len < 0) | (len > maxp32));
        send = TERM | (bad ? TBAD : 0) | (ts + c);
      } else if (nx >= FT_S) {
        send = ts + nx;
        if (lane == 0) ft_mark_exit(xbits, nx - FT_S, W);
      } else {
        send = TERM | (ts + nx);             // the stream ends at nx
      }
    }
    if (lane < (m & 63)) L[(m & ~63) + lane] = (uint16_t)ent;
    // survivor bit map for the join walk, from the list just stored (each
    // lane rereads only the entries it wrote itself)
    for (int i = lane; i < m; i += 64) {
      const int32_t q = L[i];
      __hip_atomic_fetch_or(&sbits[q >> 5], 1u << (q & 31), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
  }
  // ---- 3. publish this tile's exit candidates; take the tile before's -----
  // preferred candidate: the survivor's exit, else the latest in-window
  // exit of the frontier (-1: none)
  int32_t px = -1;
  // (LONG: the survivor's exit may lie past the window — after a frame
  // longer than the window the chain resumes there, and the next tile's
  // frontier passes find it)
  if (sm && !(send & TERM) && send - tend < (LONG ? FT_S - 1 : W)) {
    px = (int32_t)(send - tend);
  } else {
    uint32_t lx = lastx;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1)
      lx = max(lx, (uint32_t)__shfl_xor((int)lx, d, 64));
    if (lx != 0) px = (int32_t)(lx & 0xFFFF);
  }
  // Candidates go out packed in ONE 64-bit word (a relaxed agent-scope
  // store, like the single exit before: no fence, no L2 write-back on this
  // multi-XCD part): bit 63 = ready, five 12-bit slots of offset + 1
  // (0 = empty), slot 0 the preferred one, then up to four other in-window
  // exits in offset order.
  __builtin_amdgcn_wave_barrier();
  uint64_t word = (uint64_t)1 << 63;
  if (px >= 0) word |= (uint64_t)(px + 1);
  {
    uint32_t xw = lane < XW ? xbits[lane] : 0u;
    if (px >= 0 && lane == (px >> 5)) xw &= ~(1u << (px & 31));
    uint64_t any = __ballot(xw != 0);
    int slot = 1;
    while (any && slot < 5) {
      const int wl = (int)__builtin_ctzll(any);
      uint32_t bits = (uint32_t)__builtin_amdgcn_readlane((int)xw, wl);
      while (bits && slot < 5) {
        const int bit = (int)__builtin_ctz(bits);
        bits &= bits - 1;
        word |= (uint64_t)(wl * 32 + bit + 1) << (12 * slot);
        ++slot;
      }
      any &= any - 1;
    }
  }
  if (lane == 0) lb_store(&lbw[2 * t], word);    // 0 = not yet
  const int64_t t_1 = dbg ? wall_clock64() : 0;
  int64_t E = 0;
  bool none = false;
  if (t > 0 && nospec) {
    // (tests: every tile but the first without a speculated entry, the
    // worst case of the link repair; no candidate exits either)
    none = true;
    if (lane < 5) cx[5 * t + lane] = FC_DEAD;
  } else if (t > 0) {
    // Tile t-1 is running or done.  Poll with exponential back-off: these
    // loads bypass the caches, and thousands of waves polling every few
    // hundred cycles flood the fabric (it tripled every tile's staging
    // latency before the back-off).
    uint64_t x;
    int nap = 0;
    const uint64_t t_w = wall_clock64();
    for (;;) {
      x = lb_load(&lbw[2 * (t - 1)]);
      if (x != 0) break;
      if (wall_clock64() - t_w > FT_WAIT_TICKS) break;   // no speculation
      switch (nap) {                        // s_sleep takes an immediate
        case 0: __builtin_amdgcn_s_sleep(2); break;
        case 1: __builtin_amdgcn_s_sleep(4); break;
        case 2: __builtin_amdgcn_s_sleep(8); break;
        case 3: __builtin_amdgcn_s_sleep(16); break;
        default: __builtin_amdgcn_s_sleep(32); break;
      }
      ++nap;
    }
    // Pick the entry among the candidates (the tile before's exits that
    // land here).  A wrong one is a garbage chain of the tile before; read
    // on in THIS tile it almost always dies on a bad length within a few
    // hops, while the true chain lives on.  Every candidate is walked (LDS
    // only, no recording) to where it leaves the tile — meeting the
    // survivor's path counts as leaving with the survivor — and the first
    // that survives is the entry.  The exits of all of them go to `cx`:
    // where two chains both survive tile after tile (a phantom chain: in
    // the storm's create replies, zxids 0x2Exxxx make the bytes 10 past
    // each frame start read as the frame length 46), the tile cannot tell
    // which is true, and fs_link's chase follows the exact one through
    // this map instead of re-walking every tile.
    E = -1;
    int64_t first = -1;
    for (int slot = 0; slot < 5; ++slot) {
      const int32_t v = (int32_t)((x >> (12 * slot)) & 0xFFF);
      int64_t xe = FC_DEAD;
      if (v != 0 && ts + (v - 1) < n) {
        const int32_t e = v - 1;
        if (first < 0) first = ts + e;
        xe = ft_cand(sb, sbits, e, nrel, maxp32, send, n, ts, m, lane);
        if (E < 0 && xe != FC_DEAD) E = ts + e;
      }
      if (lane == 0) cx[5 * t + slot] = xe;
    }
    if (E < 0) E = first;        // no live candidate: the first one
    // (tests: every misspec-th tile takes a garbage entry one byte past the
    // chosen one, the link repair's adversary)
    if (misspec > 0 && t % misspec == 1 && E >= 0 && E + 1 < n) ++E;
    none = E < 0;
  }
  const int64_t t_2 = dbg ? wall_clock64() : 0;
  // ---- 4. join: walk from the entry until the survivor's path -------------
  FcWalk w{E, 0, 0, -1, false, false};
  if (!none) {
    int64_t c = E;
    uint16_t* P = pre + t * FT_LMAX;
    int32_t np = 0;
    uint32_t ent = 0;
    for (;;) {
      if (c >= tend) { w.exit = c; break; }
      if (c >= n) { w.exit = n; break; }    // the stream ends cleanly
      const int32_t crel = (int32_t)(c - ts);
      // both LDS reads of the hop issued together (the survivor map word
      // and the length word); the map is all zero when m == 0
      const uint32_t smw = sbits[crel >> 5];
      const int32_t lraw = lds_be32(sb, crel);
      if ((smw >> (crel & 31)) & 1u) {
        // joined: the rest is the survivor's list from this start on; its
        // index is the number of survivor starts below crel (the map has
        // FT_BITS = 2 x 64 words, two per lane)
        static_assert(FT_BITS == 2 * 64, "two map words per lane");
        const int32_t cw = crel >> 5;
        int32_t s = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int32_t wi = lane + 64 * h;
          const uint32_t wd = sbits[wi];
          s += wi < cw ? __popc(wd)
                       : (wi == cw ? __popc(wd & ((1u << (crel & 31)) - 1u))
                                   : 0);
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
        w.js = s;
        break;
      }
      const int32_t len = __builtin_amdgcn_readfirstlane(lraw);
      const int32_t nx = crel + 4 + len;
      if ((uint32_t)len > (uint32_t)maxp32 || nx > nrel) {
        w.exit = c;
        w.term = true;
        w.bad = (crel + 4 <= nrel) && ((len < 0) | (len > maxp32));
        break;
      }
      ft_record(P, np, ent, crel, lane);
      c = ts + nx;
    }
    if (lane < (np & 63)) P[(np & ~63) + lane] = (uint16_t)ent;
    w.np = np;
    w.cnt = np;
    if (w.js >= 0) {
      w.cnt = np + (m - w.js);
      fc_join_end(w, send, n);
    }
  } else {
    // no speculated entry: the exit recorded is the survivor's (the likely
    // one), so fs_link's grid repair of the NEXT tile can start from it in
    // the same round as this tile's own repair (a run of such tiles settles
    // in one round, not one tile per round)
    if (sm) fc_join_end(w, send, n);
    if (lane == 0) fc_stat(stats, 1, 1);
  }
  if (lane == 0) {
    sx[t] = send;
    rcount[t] = m;
    rec_entry[t] = none ? -1 : E;
    rec_exit[t] = w.exit;
    rec_meta[t] = fc_meta(w);
    if (dbg) {
      dbg[8 * t + 0] = t_0;
      dbg[8 * t + 1] = t_1;
      dbg[8 * t + 2] = t_2;
      dbg[8 * t + 3] = wall_clock64();
      dbg[8 * t + 4] = w.np;
      dbg[8 * t + 5] = m;
      dbg[8 * t + 6] = t_s;
      dbg[8 * t + 7] = t_f;
    }
  }
}

// ---- fs_link ---------------------------------------------------------------

// Stage [wb, wb + WIN) (zero past n) into the wave's window: all WIN/1024
// 16-byte loads of a lane issued before the first LDS write.
template <int WIN>
ZK_DEV void fc_stage(const uint8_t* __restrict__ buf, int64_t n, int64_t wb,
                     uint8_t* win, int lane) {
  constexpr int PER = WIN / 1024;
  uint4 v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int64_t g = wb + 16 * (lane + 64 * j);
    v[j] = make_uint4(0, 0, 0, 0);
    if (g + 16 <= n) {
      __builtin_memcpy(&v[j], buf + g, 16);
    } else if (g < n) {
      uint8_t* b = (uint8_t*)&v[j];
      for (int k = 0; k < 16; ++k) b[k] = g + k < n ? buf[g + k] : 0;
    }
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) *(uint4*)(win + 16 * (lane + 64 * j)) = v[j];
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// fs_tile's join walk from global memory (a repair from the exact entry E),
// through a WIN-byte LDS window (4 KiB per wave: a tile in one staging;
// block 0's serial tail: 8 KiB).
template <int WIN = FC_WIN>
ZK_DEV FcWalk fc_walk(const uint8_t* __restrict__ buf, int64_t n,
                      int64_t maxp, int64_t ts, int64_t E, const uint16_t* L,
                      int32_t m0, int64_t send, uint8_t* win, uint16_t* pre,
                      int lane) {
  FcWalk r{E, 0, 0, -1, false, false};
  const int64_t tend = ts + FT_S;
  int64_t c = E;
  int64_t wb = -(int64_t)WIN;
  int32_t lb = 0;
  uint32_t lv = lane < m0 ? (uint32_t)L[lane] : 0xFFFFFFFFu;
  int32_t np = 0;
  for (;;) {
    if (c >= tend) { r.exit = c; break; }
    if (c >= n) { r.exit = n; break; }
    const uint32_t crel = (uint32_t)(c - ts);
    if (m0 > 0) {
      const int32_t j = fc_member(crel, m0, lb, lv, lane,
                                  [&](int i) { return (uint32_t)L[i]; });
      if (j >= 0) { r.js = j; break; }
    }
    if (c + 4 > n) { r.exit = c; r.term = true; break; }
    if (c < wb || c + 8 > wb + WIN) {
      wb = c & ~(int64_t)15;
      fc_stage<WIN>(buf, n, wb, win, lane);
    }
    const int32_t len =
        __builtin_amdgcn_readfirstlane(lds_be32(win, (int32_t)(c - wb)));
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
    fc_join_end(r, send, n);
  }
  return r;
}

// fs_link's grid: FL_B workgroups.  The usual scan (no broken link before
// the first terminal) is block 0 alone: the others return at once.  A
// repair runs in rounds over the whole grid (a fix-point): each round lists
// the broken links before the current first terminal and re-walks every
// one of them in parallel, one wave per link, from the exit of the tile
// before as it stands.  A link holds once its entry equals the exit before
// it; a tile whose speculated entry was missing or wrong but whose survivor
// is the true chain (the usual repair: a frontier wait that timed out, a
// garbage candidate that survived its tile) re-walks to the same exit, so
// one round settles any number of such tiles at once — where the serial
// repair paid one tile after the other (the round-2 storm stream: 50 ms).
// What a round cannot settle is a chain of exits that each depend on the
// previous repair (frames longer than the window crossing tile after tile):
// after FL_GROUNDS rounds block 0 finishes those serially, skipping the
// tiles a long frame covers in one step.
constexpr int FL_B = 64;                   // fs_link workgroups
constexpr int FL_GROUNDS = 6;              // grid repair rounds
constexpr uint64_t FL_BAR_TICKS = 50000000;   // 0.5 s: barrier abandoned
// grid words after lbw's stats (uint64): [0] barrier arrivals, [1] barrier
// generation, [2] abort, then per round r [4 + 2r] broken links listed (the
// chase repair, which runs no rounds, uses [3] settled and [5] / [6] its
// grid check's first broken link / terminal)
constexpr int FL_NB = 3 + 2 * FL_GROUNDS;     // broken links fs_check saw
constexpr int FL_GW = FL_NB + 1;
// At most this many broken links: chased from fs_check's list (fl_chase; a
// reply stream usually has a handful of broken links or none); more (every
// tile without a speculated entry) go to the grid rounds.
constexpr unsigned long long FL_SMALL = 1024;

// Grid barrier over fs_link's FL_B workgroups (they are co-resident: 64
// blocks on a 256-CU part, and nothing they wait for needs a CU they hold).
// Every wait is bounded: past FL_BAR_TICKS the grid is told to abort and
// block 0 falls back to the serial repair.  Returns false on abort.
ZK_DEV bool fl_sync(unsigned long long* g) {
  __shared__ int s_ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = 1;
    __threadfence();
    const unsigned long long gen =
        __hip_atomic_load(&g[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long a =
        __hip_atomic_fetch_add(&g[0], 1ull, __ATOMIC_ACQ_REL,
                               __HIP_MEMORY_SCOPE_AGENT) + 1;
    if (a == gridDim.x) {
      __hip_atomic_store(&g[0], 0ull, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&g[1], 1ull, __ATOMIC_RELEASE,
                             __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint64_t t0 = wall_clock64();
      while (__hip_atomic_load(&g[1], __ATOMIC_ACQUIRE,
                               __HIP_MEMORY_SCOPE_AGENT) == gen) {
        if (__hip_atomic_load(&g[2], __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT)) {
          ok = 0;
          break;
        }
        if (wall_clock64() - t0 > FL_BAR_TICKS) {
          __hip_atomic_store(&g[2], 1ull, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(8);
      }
    }
    __threadfence();
    if (__hip_atomic_load(&g[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      ok = 0;
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

// Is a repair walk of tile k (new exit x) written?  Always when the link
// before k holds (its entry E is then exact, or at least as good as the
// records get).  When that link is itself broken, E is suspect: a garbage
// exit of tile k-1 (say a frame-length read from an xid, megabytes ahead)
// walked on would break the link after k where it holds, that link's walk
// would break the next, and a wave of garbage would cross the stream one
// tile per round, with the true repair one round behind it (the first storm
// reply stream: 1413 tiles re-walked over 71 rounds).  So a suspect walk
// that changes the exit is not written while link k+1 holds; link k stays
// broken and is walked again once the tile before has settled.  The
// leftmost broken link always has an exact entry, so every round settles
// at least it.  A walk from an E that tile k-1 has since replaced is stale
// and not written either.  (A refused walk has overwritten the tile's
// recorded frame starts all the same: its caller clears the entry.)
ZK_DEV bool fl_accept(const int64_t* rec_entry, const int64_t* rec_exit,
                      int64_t ntiles, int64_t k, int64_t E, int64_t x) {
  if (ld_agent(&rec_exit[k - 1]) != E) return false;
  if (k < 2) return true;
  const bool suspect = ld_agent(&rec_entry[k - 1]) != ld_agent(&rec_exit[k - 2]);
  if (!suspect) return true;
  const int64_t ox = ld_agent(&rec_exit[k]);
  if (x == ox || k + 1 >= ntiles) return true;
  return ld_agent(&rec_entry[k + 1]) != ox;
}

// One grid repair round (every thread of every block calls it).  Returns
// false when no link was broken (the fix-point is reached) or on abort.
ZK_DEV bool fl_round(const uint8_t* __restrict__ buf, int64_t n,
                     int64_t ntiles, int64_t maxp,
                     const int64_t* __restrict__ sx,
                     const uint16_t* __restrict__ list,
                     const int32_t* __restrict__ rcount, uint16_t* pre,
                     int64_t* rec_entry, int64_t* rec_exit, int64_t* rec_meta,
                     int32_t* blist, unsigned long long* g, int r,
                     int64_t* red, uint8_t* win, uint64_t* stats) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t INF = INT64_MAX;
  const int64_t nblk = gridDim.x;
  const int64_t bid = blockIdx.x;
  const int64_t nth = nblk * FL_T;
  const int64_t gt = bid * FL_T + tid;
  // B. list the broken links (after a tile that is not a terminal).  Every
  // one, not only those before the first terminal: a terminal may be a
  // speculation's (a garbage entry that died) that this very round fixes,
  // and stopping the list there made a stream with many such tiles take a
  // round per terminal (26 ms a 0-1024 B reply stream at a 1 KiB window).
  // Past a real bad frame the walks are wasted, and the serial tail's
  // first terminal bounds what counts.
  int64_t nb = 0;
  const int64_t per = (ntiles - 1 + nth - 1) / nth;
  const int64_t k0 = 1 + gt * per, k1 = min(k0 + per, ntiles);
  auto broken = [&](int64_t k) {
    return ld_agent(&rec_entry[k]) != ld_agent(&rec_exit[k - 1]) &&
           !m_term(ld_agent(&rec_meta[k - 1]));
  };
  for (int64_t k = k0; k < k1; ++k) nb += broken(k);
  int64_t tot;
  const int64_t o = block_excl_scan(nb, red, &tot);
  __shared__ unsigned long long s_base;
  if (tid == 0)
    s_base = tot ? atomicAdd(&g[4 + 2 * r], (unsigned long long)tot) : 0;
  __syncthreads();
  int64_t w = (int64_t)s_base + o;
  for (int64_t k = k0; k < k1; ++k)
    if (broken(k)) blist[w++] = (int32_t)k;
  if (!fl_sync(g)) return false;
  const int64_t nbr = (int64_t)__hip_atomic_load(
      &g[4 + 2 * r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (nbr == 0) return false;
  // C. every listed link re-walked by one wave, from the exit before it
  uint8_t* mywin = win + (size_t)wv * (FC_WIN + 16);
  const int64_t nwv = nblk * (FL_T / 64);
  uint32_t walked = 0;
  for (int64_t j = bid * (FL_T / 64) + wv; j < nbr; j += nwv) {
    const int64_t k = blist[j];
    const int64_t E = ld_agent(&rec_exit[k - 1]);
    if (E < k * FT_S) continue;               // no exact entry yet
    const int32_t m0 = __builtin_amdgcn_readfirstlane(rcount[k]);
    const FcWalk fw = fc_walk(buf, n, maxp, k * FT_S, E, list + k * FT_LMAX,
                              m0, sx[k], mywin, pre + k * FT_LMAX, lane);
    ++walked;
    if (lane == 0) {
      if (fl_accept(rec_entry, rec_exit, ntiles, k, E, fw.exit)) {
        st_agent(&rec_entry[k], E);
        st_agent(&rec_exit[k], fw.exit);
        st_agent(&rec_meta[k], fc_meta(fw));
      } else {
        // the walk overwrote the tile's frame starts (pre) while its
        // record keeps the old entry: no entry, so the link stays broken
        // and the tile is walked again (its exit, which the refusal
        // protects, is kept)
        st_agent(&rec_entry[k], -1);
      }
    }
  }
  if (lane == 0 && walked) fc_stat(stats, 2, walked);
  if (bid == 0 && tid == 0) fc_stat(stats, 3, 1);
  return fl_sync(g);
}

// fs_check: every link and terminal checked in parallel (one thread per
// tile, a grid over the tiles) and the frame counts scanned per block of
// FK_T tiles: base[k] = count before tile k within its block, bsum[b] = the
// block's total.  The leftmost broken link and terminal reach fs_link as
// (ntiles - k) maxima in mins[0..1] (zeroed with the X flags; one atomic
// per block).  Round 2's fs_link did this in one workgroup, ~25 dependent
// round trips per thread on a 100 MB stream (60 us per scan).
constexpr int FK_T = 256;
__global__ __launch_bounds__(FK_T) void fs_check(
    const int64_t* __restrict__ n_dev, int64_t n_cap,
    const int64_t* __restrict__ rec_entry, const int64_t* __restrict__ rec_exit,
    const int64_t* __restrict__ rec_meta, int64_t* __restrict__ base,
    int64_t* __restrict__ bsum, uint64_t* __restrict__ mins,
    unsigned long long* __restrict__ nbroken, int32_t* __restrict__ blist) {
  __shared__ int64_t sm[FK_T / 64 + 1];
  __shared__ int64_t smin[2 * (FK_T / 64)];
  const int64_t n = stream_len(n_dev, n_cap);
  const int64_t ntiles = (n + FT_S - 1) / FT_S;
  const int64_t k = (int64_t)blockIdx.x * FK_T + threadIdx.x;
  if ((int64_t)blockIdx.x * FK_T >= ntiles) return;       // block-uniform
  const int64_t INF = INT64_MAX;
  int64_t cnt = 0, fb = INF, fterm = INF;
  if (k < ntiles) {
    // written by fs_tile (an earlier launch): plain loads, issued together
    const int64_t mk = rec_meta[k];
    const bool nxt = k + 1 < ntiles;
    const int64_t e = nxt ? rec_entry[k + 1] : 0;
    const int64_t x = rec_exit[k];
    cnt = m_cnt(mk);
    if (m_term(mk)) fterm = k;
    else if (nxt && (e < 0 || e != x)) fb = k + 1;
  }
  // broken links, counted and listed (fs_link picks its repair by the
  // count; a small repair starts from the list)
  const uint64_t bm = __ballot(fb != INF);
  if (bm) {
    const int lane = threadIdx.x & 63;
    unsigned long long b0 = 0;
    if (lane == 0) b0 = atomicAdd(nbroken, (unsigned long long)__popcll(bm));
    b0 = __shfl(b0, 0, 64);
    if (fb != INF) {
      const uint64_t below = lane ? (bm & ((~0ull) >> (64 - lane))) : 0ull;
      blist[b0 + __popcll(below)] = (int32_t)fb;
    }
  }
  int64_t tot;
  const int64_t ex = block_excl_scan(cnt, sm, &tot);
  if (k < ntiles) base[k] = ex;
  for (int d = 32; d >= 1; d >>= 1) {
    fb = min(fb, (int64_t)__shfl_xor(fb, d, 64));
    fterm = min(fterm, (int64_t)__shfl_xor(fterm, d, 64));
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smin[wv] = fb;
    smin[FK_T / 64 + wv] = fterm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int j = 1; j < FK_T / 64; ++j) {
      fb = min(fb, smin[j]);
      fterm = min(fterm, smin[FK_T / 64 + j]);
    }
    bsum[blockIdx.x] = tot;
    if (fb != INF) atomicMax((unsigned long long*)&mins[0],
                             (unsigned long long)(ntiles - fb));
    if (fterm != INF) atomicMax((unsigned long long*)&mins[1],
                                (unsigned long long)(ntiles - fterm));
  }
}

// Row bases once every link up to the first terminal ft (INF: none) holds:
// bsum[b] (block b's count total, fs_check's or re-counted) becomes block
// b's exclusive offset; base[k] stays the in-block one; result[0..3] and
// the last tile.  Block 0 alone.
ZK_DEV void fl_bases(int64_t n, int64_t ntiles, int64_t ft,
                     const int64_t* rec_exit, const int64_t* rec_meta,
                     const int64_t* base, int64_t* bsum, int64_t cap,
                     int64_t* result, int64_t* lastk, int64_t* red) {
  const int tid = threadIdx.x;
  const int64_t INF = INT64_MAX;
  const int64_t last = ft == INF ? ntiles - 1 : ft;
  const int64_t nbl = last / FK_T + 1;
  const int64_t per = (nbl + FL_T - 1) / FL_T;
  const int64_t b0 = (int64_t)tid * per;
  const int64_t b1 = min(b0 + per, nbl);
  int64_t sum = 0;
  for (int64_t b = b0; b < b1; ++b) sum += ld_agent(&bsum[b]);
  int64_t tot;
  int64_t run = block_excl_scan(sum, red, &tot);
  const int64_t blast = last / FK_T;
  for (int64_t b = b0; b < b1; ++b) {
    const int64_t v = ld_agent(&bsum[b]);
    bsum[b] = run;
    if (b == blast) {
      // frames up to `last` (tiles after it in its block are dead)
      const int64_t ml = ld_agent(&rec_meta[last]);
      const int64_t total = run + ld_agent(&base[last]) + m_cnt(ml);
      *lastk = last;
      result[0] = total;
      result[3] = total > cap ? 1 : 0;
      if (ft == INF) {
        result[1] = n;
        result[2] = 0;
      } else {
        result[1] = ld_agent(&rec_exit[ft]);
        result[2] = m_bad(ml) ? 1 : 0;
      }
    }
    run += v;
  }
}

// The small repair (a handful of broken links, the usual kind): CHASES.
// fs_check listed the broken links.  A chase starts at one with the exact
// entry (the exit before it) and runs forward while the link after the
// tile it settled is still broken.  Most tiles of a run need no walk:
// their exact entry is one of the candidate entries fs_tile walked, whose
// exit and frame count `cx` already holds (fs_tile's entry -> exit map),
// so the chase only looks it up — a wave loads the candidate words and
// exits of 64 tiles at once and resolves them with a 6-step parallel
// prefix over the tiles' slot maps.  A tile whose entry is not a candidate
// (a frame longer than the window) is walked; tiles a long frame covers
// whole are filled in one step.  Looked-up tiles are marked stale: fs_rows
// walks their frame starts, in parallel with every other tile.  (Round 3
// first re-walked every tile of a run one after the other: on the storm's
// phantom-chain replies, 650 tiles in 18 ms; then looked them up one tile
// at a time, ~0.3 us each.)
// Chases of different runs run in parallel (one wave each) in rounds: a
// round's chases, then a check of every run's first and last link (another
// run may have moved an exit), the broken ones (deduplicated in an LDS
// hash set) chased next round.  Only the count blocks holding a re-written
// tile are re-counted.  When the lists outgrow LDS or the rounds run out,
// block 0's serial tail finishes from the records as they stand.
constexpr int FL_WL = 1024;                // chases per round
constexpr int FL_HS = 2048;                // their dedup hash set
constexpr int FL_WR = 48;                  // rounds before the serial tail
constexpr int FL_DB = 8192;                // count blocks tracked (2M tiles)
static_assert(FL_SMALL <= FL_WL, "fs_check's list fits the first round");

struct FlChase {
  uint32_t* dirty;                // count blocks holding re-written tiles
  int* overflow;
  uint64_t* stats;
  int64_t* clk;                   // ZKMI_FS_DBG: the exact chase's span
};

ZK_DEV void fl_dirty(FlChase& ch, int64_t t) {
  const int64_t b = t / FK_T;
  atomicOr(&ch.dirty[b >> 5], 1u << (b & 31));
}

ZK_DEV int live_count(const int64_t* c5) {
  int live = 0;
#pragma unroll
  for (int j = 0; j < 5; ++j) live += c5[j] != FC_DEAD;
  return live;
}

ZK_DEV int64_t rfl64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

ZK_DEV uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// One chase (one wave) from broken link k0.  Returns the last tile it
// wrote (-1: none), `term` when that tile ends the chain.
// `exact`: k0 is the round's leftmost broken link, so its entry (the exit
// before it) is exact and so is everything the chase derives.  It stops at
// a link that holds only where the tile after is unambiguous (one live
// candidate): a run of tiles where two chains both survive (a phantom
// chain) can hold links that are consistent and wrong, and only a chase
// from an exact entry can tell — it goes through the whole run.
// Otherwise (another broken link of the round, entry not known exact) the
// chase writes nothing that would break a link that holds (fl_accept's
// rule: a phantom's exit must not run over a true segment); it stops there
// and the link waits for a later round.
ZK_DEV int64_t fl_chase_run(const uint8_t* __restrict__ buf, int64_t n,
                            int64_t ntiles, int64_t maxp,
                            const int64_t* __restrict__ sx,
                            const uint16_t* __restrict__ list,
                            const int32_t* __restrict__ rcount, uint16_t* pre,
                            int64_t* rec_entry, int64_t* rec_exit,
                            int64_t* rec_meta, const uint64_t* lbw,
                            const int64_t* cx,
                            uint8_t* mywin, FlChase& ch, int64_t k0,
                            bool exact, bool& term, uint32_t& walked) {
  const int lane = threadIdx.x & 63;
  term = false;
  // everything that steers the chase is wave-uniform; saying so keeps its
  // control flow scalar (else the compiler runs the batch loop below as
  // divergent code under exec masks: ~850 cycles a tile)
  k0 = rfl64(k0);
  exact = __builtin_amdgcn_readfirstlane((int)exact) != 0;
  int64_t k = k0;
  int64_t E = rfl64(ld_agent(&rec_exit[k - 1]));
  if (E < k * FT_S ||
      __builtin_amdgcn_readfirstlane(m_term(ld_agent(&rec_meta[k - 1]))))
    return -1;
  if (!exact && rfl64(ld_agent(&rec_entry[k])) == E) return -1;  // holds
  bool first = true;             // tile k0's own link is the broken one
  for (;;) {
    if (E >= (k + 1) * FT_S) {
      // a frame covers tiles k .. kx-1 whole: no frame starts there.  (Only
      // from an exact entry: a garbage exit megabytes ahead would wipe out
      // every tile it claims to cover.)
      if (!exact) return k - 1;
      const int64_t kend = min(E / FT_S, ntiles);
      const FcWalk cov{E, 0, 0, -1, false, false};
      for (int64_t c = k + lane; c < kend; c += 64) {
        st_agent(&rec_entry[c], E);
        st_agent(&rec_exit[c], E);
        st_agent(&rec_meta[c], fc_meta(cov));
        fl_dirty(ch, c);
      }
      if (kend >= ntiles) return kend - 1;
      k = kend;
      first = false;
      continue;
    }
    // ---- a batch of 64 tiles, lane i = tile k+i ------------------------
    // Each lane loads its tile's candidate word (written by the tile
    // before), the five candidate exits, its entry and exit and the next
    // tile's entry, and turns them into a transition table over its five
    // candidate slots: the slot of the next tile that each exit enters
    // (next lane's word), whether the link into this tile holds with that
    // slot's entry, whether taking it would break a holding link, whether
    // two candidates survive.  The serial walk over the batch is then a
    // few scalar instructions a tile.  (Round 3 first resolved each tile
    // from the raw words: ~150 dependent instructions, 0.6 us a tile.)
    const int64_t tl = k + lane;
    const int64_t ts_l = tl * FT_S;
    uint64_t wd = 0;
    int64_t en = INT64_MIN, ent = INT64_MIN, ox = INT64_MIN + 1;
    int64_t c5[5];               // candidate exits
    int32_t n5[5];               // and their frame counts
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      c5[j] = FC_DEAD;
      n5[j] = 0;
    }
    if (tl < ntiles) {
      wd = lb_load(&lbw[2 * (tl - 1)]);
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const int64_t v = cx[5 * tl + j];
        c5[j] = cx_exit(v);
        n5[j] = cx_cnt(v);
      }
      ent = ld_agent(&rec_entry[tl]);
      ox = ld_agent(&rec_exit[tl]);
    }
    if (tl + 1 < ntiles) en = ld_agent(&rec_entry[tl + 1]);
    // the next tile's slots
    const uint32_t wn_lo = (uint32_t)__shfl_down((int)(uint32_t)wd, 1, 64);
    const uint32_t wn_hi =
        (uint32_t)__shfl_down((int)(uint32_t)(wd >> 32), 1, 64);
    const uint64_t wn = ((uint64_t)wn_hi << 32) | wn_lo;
    const int64_t tend_l = ts_l + FT_S;
    const bool next_holds = tl + 1 < ntiles && en == ox;
    // lane i's map M over the state of its tile — the entry slot 0..4, or
    // 5 stopped (an earlier tile ended the run), 6 walk (the entry is the
    // exit before, not among the candidates), 7 leave (the entry lies
    // past the tile or the batch) — to the state of the tile after it.
    // Tile i stops the run (maps to 5) when its link already holds with
    // that entry (an exact chase goes on through ambiguous tiles), when a
    // non-exact chase would break a holding link, or when the exit is not
    // known (the tile is walked).
    const bool amb = live_count(c5) >= 2;
    const bool head = first && lane == 0;   // k0: its link is the broken one
    uint32_t M = (5u << 15) | (5u << 18) | (5u << 21);
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const uint32_t oj = (uint32_t)((wd >> (12 * j)) & 0xFFF);  // off + 1
      const int64_t xj = c5[j];
      uint32_t nx = 5;                      // (no looked-up exit: stops)
      if (tl < ntiles && oj != 0 && xj >= tend_l) {
        if (xj >= tend_l + FT_S || lane == 63 || tl + 1 >= ntiles) {
          nx = 7;
        } else {
          const uint32_t want = (uint32_t)(xj - tend_l) + 1;
          nx = 6;
#pragma unroll
          for (int q = 4; q >= 0; --q)
            if ((uint32_t)((wn >> (12 * q)) & 0xFFF) == want) nx = q;
        }
        const bool holds = ent == ts_l + (int64_t)oj - 1;
        if (!head && holds && !(exact && amb)) nx = 5;
        if (!exact && xj != ox && next_holds) nx = 5;
      }
      M |= nx << (3 * j);
    }
    // the state of the batch's first tile
    uint32_t j0 = 6;
    {
      const uint64_t w0 = readlane64(wd, 0);
      const uint32_t want = (uint32_t)(E - k * FT_S) + 1;
#pragma unroll
      for (int q = 4; q >= 0; --q)
        if ((uint32_t)((w0 >> (12 * q)) & 0xFFF) == want) j0 = q;
    }
    // prefix composition over the lanes (Hillis-Steele, 6 steps): T_i =
    // M_i o ... o M_0; the state of tile i is T_{i-1}(j0)
    uint32_t T = M;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t U = (uint32_t)__shfl_up((int)T, d, 64);
      if (lane >= d) {
        uint32_t C = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q)
          C |= ((T >> (3 * ((U >> (3 * q)) & 7))) & 7) << (3 * q);
        T = C;
      }
    }
    const uint32_t Tp = (uint32_t)__shfl_up((int)T, 1, 64);
    const uint32_t st = lane == 0 ? j0 : (Tp >> (3 * j0)) & 7;
    // looked up: a tile whose state is an entry slot and whose map does not
    // stop there
    const bool mine = tl < ntiles && st < 5 && ((M >> (3 * st)) & 7) != 5;
    const uint64_t looked = __ballot(mine);
    // the run of looked-up tiles is a prefix of the batch
    const int f = looked == ~0ull ? 64 : (int)__builtin_ctzll(~looked);
    if (f > 0) {
      if (lane == 0) fc_stat(ch.stats, 0, (uint32_t)f);
      if (lane < f) {
        // exact entry, exit and frame count; the frame starts themselves
        // are walked by fs_rows (a stale tile)
        const uint32_t oj = (uint32_t)((wd >> (12 * st)) & 0xFFF);
        const int64_t xj = st == 0 ? c5[0] : st == 1 ? c5[1]
                           : st == 2 ? c5[2] : st == 3 ? c5[3] : c5[4];
        const int32_t nj = st == 0 ? n5[0] : st == 1 ? n5[1]
                           : st == 2 ? n5[2] : st == 3 ? n5[3] : n5[4];
        st_agent(&rec_entry[tl], ts_l + (int64_t)oj - 1);
        st_agent(&rec_exit[tl], xj);
        st_agent(&rec_meta[tl], M_STALE | nj);
        fl_dirty(ch, tl);
      }
      first = false;
    }
    if (k + f >= ntiles) return ntiles - 1;
    // what ends the run at tile k+f: its state
    const uint32_t sf = (uint32_t)__builtin_amdgcn_readlane((int)st, f & 63);
    if (f < 64 && sf < 5) {
      // its map stops there: the link holds, a refusal, or no known exit
      const uint32_t oj = (uint32_t)((readlane64(wd, f) >> (12 * sf)) & 0xFFF);
      const int64_t xs = (int64_t)readlane64(
          (uint64_t)(sf == 0 ? c5[0] : sf == 1 ? c5[1] : sf == 2 ? c5[2]
                     : sf == 3 ? c5[3] : c5[4]), f);
      if (xs >= (k + f + 1) * FT_S) return k + f - 1;   // link / refusal
      E = (k + f) * FT_S + (int64_t)oj - 1;              // walked below
    } else {
      // 6 / 7 (or the batch done): the entry is the exit before it
      const int l = f - 1;
      const uint32_t sl =
          (uint32_t)__builtin_amdgcn_readlane((int)st, l < 0 ? 0 : l);
      if (l >= 0)
        E = (int64_t)readlane64(
            (uint64_t)(sl == 0 ? c5[0] : sl == 1 ? c5[1] : sl == 2 ? c5[2]
                       : sl == 3 ? c5[3] : c5[4]), l);
    }
    k += f;
    if (f == 64 || sf == 7) continue;          // next batch / covered

    // stop == 2: tile k (entry E) is walked
    {
      const int64_t t = k;
      if (t >= ntiles) return t - 1;
      if (E >= (t + 1) * FT_S) continue;          // covered: to the top
      if (!first && rfl64(ld_agent(&rec_entry[t])) == E && !exact)
        return t - 1;
      const int64_t ts = t * FT_S;
      const int64_t oldx = rfl64(ld_agent(&rec_exit[t]));
      const bool nh = t + 1 < ntiles &&
                      rfl64(ld_agent(&rec_entry[t + 1])) == oldx;
      const int32_t m0 = __builtin_amdgcn_readfirstlane(rcount[t]);
      const FcWalk fw = fc_walk(buf, n, maxp, ts, E, list + t * FT_LMAX, m0,
                                sx[t], mywin, pre + t * FT_LMAX, lane);
      ++walked;
      if (!exact && rfl64(fw.exit) != oldx && nh) {
        // refused, but the walk overwrote the tile's frame starts: no
        // entry, so its link stays broken (see fl_round)
        if (lane == 0) st_agent(&rec_entry[t], -1);
        return t - 1;
      }
      if (lane == 0) {
        st_agent(&rec_entry[t], E);
        st_agent(&rec_exit[t], fw.exit);
        st_agent(&rec_meta[t], fc_meta(fw));
        fl_dirty(ch, t);
      }
      first = false;
      if (__builtin_amdgcn_readfirstlane(fw.term)) { term = true; return t; }
      if (t + 1 >= ntiles) return t;
      // an exact chase stops where the next link holds and the tile after
      // has one live candidate; the next batch checks that
      E = rfl64(fw.exit);
      k = t + 1;
    }
  }
}

// Block 0: chase rounds to a fix-point of the links.  Returns false when it
// gave up (the serial tail takes over).
ZK_DEV bool fl_chase(const uint8_t* __restrict__ buf, int64_t n,
                     int64_t ntiles, int64_t maxp,
                     const int64_t* __restrict__ sx,
                     const uint16_t* __restrict__ list,
                     const int32_t* __restrict__ rcount, uint16_t* pre,
                     int64_t* rec_entry, int64_t* rec_exit, int64_t* rec_meta,
                     const uint64_t* lbw, const int64_t* cx, int32_t* blist,
                     int nb0, uint8_t* win, uint64_t* stats, FlChase& ch) {
  __shared__ int32_t wl[2][FL_WL];
  __shared__ int32_t wk[FL_WL];              // run ends (+ 1; 0: none)
  __shared__ uint32_t hs[FL_HS];
  __shared__ int s_n;
  __shared__ int s_cur;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // fs_check's list to LDS
  for (int i = tid; i < nb0; i += FL_T) wl[0][i] = blist[i];
  if (tid == 0) s_cur = nb0;
  uint8_t* mywin = win + (size_t)wv * (FC_WIN + 16);
  int cur = 0, rounds = 0;
  uint32_t walked = 0;
  __syncthreads();
  int ncur = s_cur;
  while (ncur > 0) {
    if (rounds == FL_WR) break;
    ++rounds;
    const int nxt = cur ^ 1;
    for (int i = tid; i < FL_HS; i += FL_T) hs[i] = 0;
    if (tid == 0) s_n = 0;
    __syncthreads();
    // one lane lists link k for the next round (once)
    auto push = [&](int64_t k) {
      const uint32_t key = (uint32_t)k + 1;
      uint32_t h = (key * 2654435761u) >> (32 - 11);
      for (;;) {
        const uint32_t old = atomicCAS(&hs[h], 0u, key);
        if (old == 0) break;
        if (old == key) return;
        h = (h + 1) & (FL_HS - 1);
      }
      const int i = atomicAdd(&s_n, 1);
      if (i < FL_WL) wl[nxt][i] = (int32_t)k;
      else *ch.overflow = 1;
    };
    // the round's leftmost broken link: its entry is exact
    int32_t lo = INT32_MAX;
    for (int j = lane; j < ncur; j += 64) lo = min(lo, wl[cur][j]);
    for (int d = 32; d >= 1; d >>= 1) lo = min(lo, __shfl_xor(lo, d, 64));
    for (int j = wv; j < ncur; j += FL_T / 64) {
      bool term;
      const bool ex = wl[cur][j] == lo;
      if (ex && ch.clk && lane == 0) ch.clk[6] = wall_clock64();
      const int64_t kend = fl_chase_run(buf, n, ntiles, maxp, sx, list,
                                        rcount, pre, rec_entry, rec_exit,
                                        rec_meta, lbw, cx, mywin,
                                        ch, wl[cur][j], wl[cur][j] == lo,
                                        term, walked);
      if (ex && ch.clk && lane == 0) ch.clk[7] = wall_clock64();
      if (lane == 0)
        wk[j] = kend < 0 ? 0 : (int32_t)(kend + 1) | (term ? (1 << 30) : 0);
    }
    __syncthreads();
    // every run's first and last link, as the records stand now
    for (int j = tid; j < ncur; j += FL_T) {
      const int64_t k0 = wl[cur][j];
      if (ld_agent(&rec_entry[k0]) != ld_agent(&rec_exit[k0 - 1]) &&
          !m_term(ld_agent(&rec_meta[k0 - 1])))
        push(k0);
      const int32_t e = wk[j];
      if (e == 0 || (e & (1 << 30))) continue;
      const int64_t kend = (e & ((1 << 30) - 1)) - 1;
      if (kend + 1 < ntiles &&
          ld_agent(&rec_entry[kend + 1]) != ld_agent(&rec_exit[kend]))
        push(kend + 1);
    }
    __syncthreads();
    if (tid == 0) s_cur = *ch.overflow ? -1 : s_n;
    __syncthreads();
    ncur = s_cur;
    cur = nxt;
    __syncthreads();
    if (ncur < 0) break;
  }
  if (lane == 0 && walked) fc_stat(stats, 2, walked);
  if (tid == 0 && rounds) fc_stat(stats, 3, rounds);
  return ncur == 0 && !*ch.overflow;
}

// After the chases and the grid's check of every link (block 0): re-count
// the count blocks holding a re-written tile, one wave per block, four
// tiles per lane.
ZK_DEV void fl_chase_recount(int64_t ntiles, const int64_t* rec_meta,
                             int64_t* base, int64_t* bsum, FlChase& ch) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nbl = (ntiles + FK_T - 1) / FK_T;
  for (int64_t b = wv; b < nbl; b += FL_T / 64) {
    if (!((ch.dirty[b >> 5] >> (b & 31)) & 1u)) continue;
    const int64_t k0 = b * FK_T + 4 * lane;
    int64_t c[4], s = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c[u] = k0 + u < ntiles ? m_cnt(ld_agent(&rec_meta[k0 + u])) : 0;
      s += c[u];
    }
    int64_t inc = s;
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t v = __shfl_up(inc, d, 64);
      if (lane >= d) inc += v;
    }
    int64_t run = inc - s;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (k0 + u < ntiles) st_agent(&base[k0 + u], run);
      run += c[u];
    }
    if (lane == 63) st_agent(&bsum[b], inc);
  }
  __syncthreads();
}

__global__ __launch_bounds__(FL_T) void fs_link(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ n_dev,
    int64_t n_cap, int64_t maxp, const int64_t* __restrict__ sx,
    const uint16_t* __restrict__ list, const int32_t* __restrict__ rcount,
    uint16_t* pre, int64_t* rec_entry, int64_t* rec_exit, int64_t* rec_meta,
    int64_t* __restrict__ base, int64_t cap, int64_t* __restrict__ result,
    uint64_t* stats, int32_t* __restrict__ blist,
    int64_t* __restrict__ bsum, uint64_t* __restrict__ mins,
    int64_t* __restrict__ lastk, unsigned long long* __restrict__ g,
    const uint64_t* lbw, const int64_t* __restrict__ cx,
    int64_t* __restrict__ ldbg) {
  __shared__ __attribute__((aligned(16)))
      uint8_t win[(FL_T / 64) * (FC_WIN + 16)];      // one per wave
  static_assert(FC_TAILWIN <= (FL_T / 64) * (FC_WIN + 16),
                "the serial tail's window is the waves' windows together");
  __shared__ int64_t red[2 * (FL_T / 64) + 2];
  __shared__ int64_t s_next;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t n = stream_len(n_dev, n_cap);
  const int64_t ntiles = (n + FT_S - 1) / FT_S;
  if (ntiles == 0) {
    if (blockIdx.x == 0) {
      if (tid < 4) result[tid] = 0;
      if (tid == 0) *lastk = -1;
    }
    return;
  }
  const int64_t INF = INT64_MAX;
  // fs_check's minima, read by every thread of every block; block 0
  // clears them for the next scan of this workspace once every block has
  // read them (on the fast path only block 0 goes on, so at once)
  const uint64_t mb0 = mins[0], mt0 = mins[1];
  const unsigned long long nb0 = g[FL_NB];
  const int64_t fb0 = mb0 ? ntiles - (int64_t)mb0 : INF;
  const int64_t ft0 = mt0 ? ntiles - (int64_t)mt0 : INF;
  const bool fast = fb0 == INF || fb0 > ft0;
  // a small repair (a handful of broken links, the usual kind) is chased
  // (fl_chase), a large one repaired in grid rounds; the whole grid takes
  // part in either (every block decides alike: block 0 clears the words it
  // read only after the grid's first barrier)
  const bool small = !fast && nb0 <= FL_SMALL &&
                     (ntiles + FK_T - 1) / FK_T <= FL_DB;
  if (fast && blockIdx.x != 0) return;
  if (fast) {
    // no broken link before the first terminal: the row bases are bsum's
    // block offsets + fs_check's in-block bases
    __syncthreads();
    if (tid == 0) {
      mins[0] = 0;
      mins[1] = 0;
      g[FL_NB] = 0;
    }
    fl_bases(n, ntiles, ft0, rec_exit, rec_meta, base, bsum, cap, result,
             lastk, red);
    return;
  }
  bool grid_ok = true;
  if (small) {
    // ---- chases: block 0; then every link checked over the grid ---------
    __shared__ uint32_t dirty[FL_DB / 32];
    __shared__ int s_ovf;
    FlChase ch{dirty, &s_ovf, stats, ldbg};
    unsigned long long* cw = &g[3];       // 1: the chases settled
    const bool clk = ldbg != nullptr && blockIdx.x == 0 && tid == 0;
    if (clk) ldbg[0] = wall_clock64();
    if (blockIdx.x == 0) {
      for (int i = tid; i < FL_DB / 32; i += FL_T) dirty[i] = 0;
      if (tid == 0) s_ovf = 0;
      __syncthreads();
      const bool ok = fl_chase(buf, n, ntiles, maxp, sx, list, rcount, pre,
                               rec_entry, rec_exit, rec_meta, lbw, cx, blist,
                               (int)nb0, win, stats, ch);
      if (tid == 0)
        __hip_atomic_store(cw, ok ? 1ull : 0ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      if (clk) ldbg[1] = wall_clock64();
    }
    bool synced = fl_sync(g);        // (block 0 cleared nothing yet)
    if (clk) ldbg[2] = wall_clock64();
    if (blockIdx.x == 0 && tid == 0) {
      mins[0] = 0;
      mins[1] = 0;
    }
    const bool settled =
        __hip_atomic_load(cw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    // every link and the first terminal, checked over the grid (a chase
    // only vouches for the links it saw): [5] / [6] = ntiles - the first
    // broken link / terminal, maxima
    if (synced) {
      const int64_t nth = (int64_t)gridDim.x * FL_T;
      int64_t fb = INF, fterm = INF;
      for (int64_t k = (int64_t)blockIdx.x * FL_T + tid; k < ntiles;
           k += nth) {
        const int64_t mk = ld_agent(&rec_meta[k]);
        if (m_term(mk)) {
          fterm = min(fterm, k);
        } else if (k + 1 < ntiles &&
                   ld_agent(&rec_entry[k + 1]) != ld_agent(&rec_exit[k])) {
          fb = min(fb, k + 1);
        }
      }
      for (int d = 32; d >= 1; d >>= 1) {
        fb = min(fb, (int64_t)__shfl_xor(fb, d, 64));
        fterm = min(fterm, (int64_t)__shfl_xor(fterm, d, 64));
      }
      if (lane == 0 && fb != INF)
        atomicMax(&g[5], (unsigned long long)(ntiles - fb));
      if (lane == 0 && fterm != INF)
        atomicMax(&g[6], (unsigned long long)(ntiles - fterm));
    }
    synced = synced && fl_sync(g);
    if (clk) ldbg[3] = wall_clock64();
    if (blockIdx.x != 0) return;
    const unsigned long long gb = __hip_atomic_load(
        &g[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long gt = __hip_atomic_load(
        &g[6], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t fbv = gb ? ntiles - (int64_t)gb : INF;
    const int64_t ftv = gt ? ntiles - (int64_t)gt : INF;
    __syncthreads();
    if (tid == 0) {
      g[2] = 0;
      g[3] = 0;
      g[5] = 0;
      g[6] = 0;
    }
    if (settled && synced && (fbv == INF || fbv > ftv)) {
      fl_chase_recount(ntiles, rec_meta, base, bsum, ch);
      if (tid == 0) g[FL_NB] = 0;
      fl_bases(n, ntiles, ftv, rec_exit, rec_meta, base, bsum, cap, result,
               lastk, red);
      if (clk) ldbg[4] = wall_clock64();
      return;
    }
    grid_ok = false;          // not settled: block 0's serial tail finishes
  } else {
    // ---- repair: rounds to a fix-point over the grid ---------------------
    grid_ok = fl_sync(g);                    // every block read the minima
    if (blockIdx.x == 0 && tid == 0) {
      mins[0] = 0;
      mins[1] = 0;
    }
  }
  for (int r = 0; r < FL_GROUNDS && grid_ok; ++r)
    grid_ok = fl_round(buf, n, ntiles, maxp, sx, list, rcount, pre,
                       rec_entry, rec_exit, rec_meta, blist, g, r, red, win,
                       stats);
  if (blockIdx.x != 0) return;
  // ---- block 0: whatever is left, serially; then the count scan -----------
  int64_t from = 1, ft = INF;
  for (;;) {
    // leftmost terminal, and leftmost broken link at or after `from`.
    // Loads in batches of FL_U tiles per thread (all issued before any is
    // used: one round trip per batch, not two per tile)
    int64_t fb = INF, fterm = INF;
    for (int64_t k0 = max(from - 1, (int64_t)0) + tid; k0 < ntiles;
         k0 += FL_U * FL_T) {
      int64_t mk[FL_U], e[FL_U], x[FL_U];
#pragma unroll
      for (int u = 0; u < FL_U; ++u) {
        const int64_t k = k0 + (int64_t)u * FL_T;
        const bool in = k < ntiles, nx = k + 1 < ntiles;
        mk[u] = in ? ld_agent(&rec_meta[k]) : 0;
        e[u] = nx ? ld_agent(&rec_entry[k + 1]) : 0;
        x[u] = in ? ld_agent(&rec_exit[k]) : 0;
      }
#pragma unroll
      for (int u = 0; u < FL_U; ++u) {
        const int64_t k = k0 + (int64_t)u * FL_T;
        if (k >= ntiles) break;
        if (m_term(mk[u])) {
          fterm = min(fterm, k);
        } else if (k + 1 < ntiles && k + 1 >= from) {
          if (e[u] < 0 || e[u] != x[u]) fb = min(fb, k + 1);
        }
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
    // terminals before from - 1 were found in an earlier pass of this loop
    // (links before `from` hold)
    if (fb == INF || fb > fterm) {          // every live link holds
      ft = fterm;
      break;
    }
    // repair: re-walk tiles from fb while their links stay broken; the
    // tiles a frame covers whole (its exit lies past them) hold no frame
    // start: they are filled in one step, not walked
    if (wv == 0) {
      int64_t k = fb;
      uint32_t walked = 0;
      for (;;) {
        const int64_t E = ld_agent(&rec_exit[k - 1]);
        const int64_t kx = E / FT_S;          // the tile the entry lies in
        if (kx > k) {
          const int64_t kend = min(kx, ntiles);
          const FcWalk cov{E, 0, 0, -1, false, false};
          for (int64_t c = k + lane; c < kend; c += 64) {
            st_agent(&rec_entry[c], E);
            st_agent(&rec_exit[c], E);
            st_agent(&rec_meta[c], fc_meta(cov));
          }
          k = kend;
          if (k >= ntiles) break;
          if (ld_agent(&rec_entry[k]) == E) break;     // link k holds
          continue;
        }
        const int32_t m0 = __builtin_amdgcn_readfirstlane(rcount[k]);
        const FcWalk w = fc_walk<FC_TAILWIN>(buf, n, maxp, k * FT_S, E,
                                             list + k * FT_LMAX, m0, sx[k],
                                             win, pre + k * FT_LMAX, lane);
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
  // the grid words back to zero for the next scan of this workspace
  if (tid < FL_GW && tid != 1) g[tid] = 0;
  // exclusive scan of the counts of tiles 0..ft; tiles after ft are dead
  const int64_t last = ft == INF ? ntiles - 1 : ft;
  const int64_t per = (last + 1 + FL_T - 1) / FL_T;
  const int64_t k0 = (int64_t)tid * per;
  const int64_t k1 = min(k0 + per, last + 1);
  int64_t sum = 0;
  for (int64_t kb = k0; kb < k1; kb += FL_U) {
    int64_t v[FL_U];
#pragma unroll
    for (int u = 0; u < FL_U; ++u)
      v[u] = kb + u < k1 ? ld_agent(&rec_meta[kb + u]) : 0;
#pragma unroll
    for (int u = 0; u < FL_U; ++u) sum += m_cnt(v[u]);
  }
  int64_t tot;
  int64_t run = block_excl_scan(sum, red, &tot);
  for (int64_t kb = k0; kb < k1; kb += FL_U) {
    int64_t v[FL_U];
#pragma unroll
    for (int u = 0; u < FL_U; ++u)
      v[u] = kb + u < k1 ? ld_agent(&rec_meta[kb + u]) : 0;
#pragma unroll
    for (int u = 0; u < FL_U; ++u) {
      if (kb + u < k1) base[kb + u] = run;
      run += m_cnt(v[u]);
    }
  }
  for (int64_t k = last + 1 + tid; k < ntiles; k += FL_T) base[k] = -1;
  // absolute bases: fs_rows adds a zero block offset
  for (int64_t b = tid; b <= last / FK_T; b += FL_T) bsum[b] = 0;
  if (tid == 0) {
    *lastk = last;
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

// (body offset, length) rows: one wave per tile, 4 tiles per block.  A
// stale tile (its exact entry, exit and count looked up by fs_link's chase)
// has no recorded frame starts for that entry: its wave stages the tile in
// LDS and walks them first.
__global__ __launch_bounds__(256) void fs_rows(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ n_dev,
    int64_t n_cap, const uint16_t* __restrict__ list,
    const uint16_t* __restrict__ pre, const int64_t* __restrict__ rec_meta,
    const int64_t* __restrict__ rec_entry,
    const int64_t* __restrict__ rec_exit,
    const int64_t* __restrict__ base, const int64_t* __restrict__ bsum,
    const int64_t* __restrict__ lastk, int64_t* __restrict__ foff,
    int32_t* __restrict__ flen, int64_t cap, uint64_t* __restrict__ lbw) {
  // (only the staged tile: 16 KiB a block keeps fs_rows at full occupancy;
  // a frame-start array beside it cost the var-size GET 3x in fs_rows)
  __shared__ __attribute__((aligned(16))) uint8_t stage[4][FT_STAGE];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t t = (int64_t)blockIdx.x * 4 + wv;
  const int64_t n = stream_len(n_dev, n_cap);
  if (t * FT_S >= n) return;
  // the scan is over for this tile: clear its candidate flags, so the next
  // scan of this workspace needs no memset (zk_frame_scan4 clean=1)
  if (lane == 0) {
    lbw[2 * t] = 0;
    lbw[2 * t + 1] = 0;
  }
  if (t > *lastk) return;
  const int64_t b = bsum[t / FK_T] + base[t];
  const int64_t m = rec_meta[t];
  const int64_t x = rec_exit[t];
  const int32_t cnt = m_cnt(m), np = m_np(m), js = m_js(m);
  const int64_t ts = t * FT_S;
  const uint16_t* P = pre + t * FT_LMAX;
  const uint16_t* R = list + t * FT_LMAX + (js < 0 ? 0 : js);
  if (m_stale(m)) {
    uint8_t* sb = stage[wv];
    fc_stage<FT_S>(buf, n, ts, sb, lane);
    if (lane == 0) {
      uint8_t* pb = sb + FT_S;
      for (int k = 0; k < 16; ++k)
        pb[k] = ts + FT_S + k < n ? buf[ts + FT_S + k] : 0;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // the walk keeps 64 starts in the lanes (lane k & 63 holds start k)
    // and writes their rows every 64 frames
    int32_t c = __builtin_amdgcn_readfirstlane((int32_t)(rec_entry[t] - ts));
    int32_t ent = 0;
    for (int32_t k = 0; k < cnt; ++k) {
      ent = lane == (k & 63) ? c : ent;
      const int32_t len = __builtin_amdgcn_readfirstlane(lds_be32(sb, c));
      c += 4 + len;
      if ((k & 63) == 63 || k == cnt - 1) {
        const int32_t last = k & 63;
        const int32_t nxt = __shfl_down(ent, 1, 64);
        if (lane <= last) {
          const int64_t p = ts + ent;
          const int64_t q = lane < last ? ts + nxt
                                        : (k == cnt - 1 ? x : ts + c);
          const int64_t idx = b + (k & ~63) + lane;
          if (idx < cap) {
            foff[idx] = p + 4;
            flen[idx] = (int32_t)(q - p - 4);
          }
        }
      }
    }
    return;
  }
  // a frame ends where the next one of the chain starts, the tile's last
  // at the tile's exit (the next tile's first frame, or the stop offset of
  // a terminal tile): lengths come from the recorded starts, no stream read
  for (int32_t k = lane; k < cnt; k += 64) {
    const int64_t p = ts + (k < np ? P[k] : R[k - np]);
    const int32_t k1 = k + 1;
    const int64_t q = k1 < cnt ? ts + (k1 < np ? P[k1] : R[k1 - np]) : x;
    const int64_t idx = b + k;
    if (idx < cap) {
      foff[idx] = p + 4;
      flen[idx] = (int32_t)(q - p - 4);
    }
  }
}

struct FsPlan {
  int64_t tiles;
  size_t off_list, off_pre, off_sx, off_lbw, off_rent, off_rexit, off_rmeta,
      off_rcnt, off_base, off_blist, off_bsum, off_cx, total;
};

static FsPlan fs_plan(int64_t n) {
  FsPlan p{};
  const int64_t tiles = n > 0 ? (n + FT_S - 1) / FT_S : 1;
  p.tiles = tiles;
  size_t o = 0;
  auto take = [&](size_t bytes) { size_t r = o; o += (bytes + 255) & ~(size_t)255; return r; };
  p.off_list = take((size_t)tiles * FT_LMAX * 2);
  p.off_pre = take((size_t)tiles * FT_LMAX * 2);
  p.off_sx = take((size_t)tiles * 8);
  // X flags (2 per tile), 4 stats words, fs_check's 2 minima, last tile,
  // a pad word, fs_link's grid words
  p.off_lbw = take((size_t)(2 * tiles + 8 + FL_GW) * 8);
  p.off_rent = take((size_t)tiles * 8);
  p.off_rexit = take((size_t)tiles * 8);
  p.off_rmeta = take((size_t)tiles * 8);
  p.off_rcnt = take((size_t)tiles * 4);
  p.off_base = take((size_t)tiles * 8);
  p.off_blist = take((size_t)tiles * 4);
  p.off_bsum = take((size_t)(tiles / FK_T + 1) * 8);
  p.off_cx = take((size_t)tiles * 5 * 8);   // candidate exits (fs_tile)
  p.total = o;
  return p;
}

// ZKMI_FS_MINB: the frontier's minimum plausible body length (default 8;
// 0 = any length, the round-2 behaviour; A/B only)
// fs_link's grid (ZKMI_FL_B, 1..FL_B, default 16): every block must find a
// CU slot before the launch ends, also on the usual path where block 0
// alone works, so a smaller grid waits less behind another stream's kernel.
static unsigned fl_blocks() {
  static int b = -1;
  if (b < 0) {
    const char* e = getenv("ZKMI_FL_B");
    b = e ? atoi(e) : 16;
    if (b < 1 || b > FL_B) b = FL_B;
  }
  return (unsigned)b;
}

static int32_t fs_minb() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ZKMI_FS_MINB");
    v = e ? atoi(e) : 8;
    if (v < 0) v = 0;
  }
  return v;
}

// scan flag: frames may be longer than the window (fs_tile's frontier
// passes past the window, and survivor exits past it as candidates)
constexpr int32_t FS_LONG = 2;

// `window` values with this bit: FS_LONG (zkmi.ops.batch.frame_window sets
// it when the window is below the stream's largest frame)
constexpr int32_t FS_WIN_LONG = 1 << 16;

static int fs_window(int32_t window) {
  window &= FS_WIN_LONG - 1;
  return window <= 256 ? 256 : window <= 512 ? 512
       : window <= 1024 ? 1024 : 2048;
}

// ZKMI_FS_DBG=1: fs_tile writes per-tile timestamps (start, survivor done,
// entry known, walk done), the walked prefix and the survivor's frame count
// into a debug buffer (zk_frame_scan_dbg copies it out).  Diagnostics only.
static int64_t* g_dbg = nullptr;
static int64_t g_dbg_tiles = 0;
static int64_t* fs_dbg_buf(int64_t tiles) {
  static int on = -1;
  if (on < 0) on = getenv("ZKMI_FS_DBG") != nullptr;
  if (!on) return nullptr;
  if (tiles > g_dbg_tiles) {
    if (g_dbg) (void)hipFree(g_dbg);
    // a row per tile (fs_tile) + one for fs_link's phase clock
    if (hipMalloc(&g_dbg, (tiles + 1) * 8 * 8) != hipSuccess) return nullptr;
    g_dbg_tiles = tiles;
  }
  return g_dbg;
}

}  // namespace zk

extern "C" {

int64_t zk_frame_scan_workspace(int64_t n) {
  return (int64_t)zk::fs_plan(n).total;
}

// K1 over buf[0, n) with n = min(*n_dev, n_cap) read ON THE DEVICE (n_dev
// null: n = n_cap): fs_tile, fs_link, fs_rows (after one memset of the
// tiles' flags).  The grids cover n_cap and tiles past n return at once, so
// a producer's device byte count (an encoder's `total`) is scanned with no
// host read and no byte past it is touched.  The launches depend only on
// n_cap, so a scan can be captured in a HIP graph and replayed over any
// length up to it.
//
// result (device int64[4]): [0] frames found, [1] stop offset (consumed
// bytes; start of the carry or of the bad frame), [2] 1 if the stop is a
// BAD_LENGTH frame, [3] 1 if the frame table overflowed `cap` (rows past
// cap are dropped).
//
// `window` (256 / 512 / 1024 / 2048 bytes) is the speculative entry window
// per 4 KiB tile: a chain can only enter a tile inside it when frames are
// <= window bytes.  Longer frames stay exact (fs_link re-walks the tiles
// after them from the exact exit, one tile at a time), so the window is a
// performance hint: the smallest one covering the stream's usual frame
// size makes the scan cheapest.  maxp must be <= 16 MiB (the protocol's
// frame limit).
// clean != 0: the workspace's flags were left cleared by the previous scan
// of it over the same n_cap (fs_rows / fs_link clear what they used), so
// the memset is skipped.  A stale flag could only cost speed, never
// correctness (fs_check / fs_link verify every speculated entry).
// flags: bit 1 (FS_LONG) frames may be longer than the window (a window
// below the stream's largest frame: fs_tile's frontier passes); tests of
// the link repair: bit 0 no speculated tile entries; bits 8..23 P > 0:
// every P-th tile (t % P == 1) takes a garbage entry.
int zk_frame_scan5(const uint8_t* buf, const int64_t* n_dev, int64_t n_cap,
                   int64_t maxp, uint8_t* ws, int64_t ws_bytes, int64_t* foff,
                   int32_t* flen, int64_t cap, int64_t* result, int32_t window,
                   int32_t clean, int32_t flags, hipStream_t st) {
  using namespace zk;
  const int W = fs_window(window);
  if (window & FS_WIN_LONG) flags |= FS_LONG;
  if (maxp > FC_MAXP || maxp < 0) return -3;
  FsPlan p = fs_plan(n_cap);
  if ((int64_t)p.total > ws_bytes) return -1;
  const int64_t tiles = p.tiles;
  uint16_t* list = (uint16_t*)(ws + p.off_list);
  uint16_t* pre = (uint16_t*)(ws + p.off_pre);
  int64_t* sx = (int64_t*)(ws + p.off_sx);
  uint64_t* lbw = (uint64_t*)(ws + p.off_lbw);
  int64_t* rent = (int64_t*)(ws + p.off_rent);
  int64_t* rexit = (int64_t*)(ws + p.off_rexit);
  int64_t* rmeta = (int64_t*)(ws + p.off_rmeta);
  int32_t* rcnt = (int32_t*)(ws + p.off_rcnt);
  int64_t* base = (int64_t*)(ws + p.off_base);
  int32_t* blist = (int32_t*)(ws + p.off_blist);
  int64_t* bsum = (int64_t*)(ws + p.off_bsum);
  int64_t* cx = (int64_t*)(ws + p.off_cx);
  uint64_t* mins = lbw + 2 * tiles + 4;
  int64_t* lastk = (int64_t*)(lbw + 2 * tiles + 6);
  unsigned long long* grid = (unsigned long long*)(lbw + 2 * tiles + 8);
  // X flags, the stats, fs_check's minima and fs_link's grid words start
  // at zero
  if (!clean &&
      hipMemsetAsync(lbw, 0, (size_t)(2 * tiles + 8 + FL_GW) * 8, st) !=
          hipSuccess)
    return -4;
  int64_t* dbg = fs_dbg_buf(tiles);
  // ZKMI_FS_TPB: tiles (waves) per block, 1..4 (A/B)
  static int tpb = -1;
  if (tpb < 0) {
    const char* e = getenv("ZKMI_FS_TPB");
    tpb = e ? atoi(e) : 4;
    if (tpb < 1 || tpb > 4) tpb = 4;
  }
  const unsigned tblocks = (unsigned)((tiles + tpb - 1) / tpb);
#define ZK_FS_TILE(WW, LL)                                                   \
  fs_tile<WW, LL><<<tblocks, 64 * tpb, FT_LDS * tpb, st>>>(                  \
      buf, n_dev, n_cap, maxp, list, pre, sx, lbw, rent, rexit, rmeta, rcnt, \
      tiles, dbg, fs_minb(), flags, cx)
  if (flags & FS_LONG) {
    switch (W) {
      case 256: ZK_FS_TILE(256, true); break;
      case 512: ZK_FS_TILE(512, true); break;
      case 1024: ZK_FS_TILE(1024, true); break;
      default: ZK_FS_TILE(2048, true); break;
    }
  } else {
    switch (W) {
      case 256: ZK_FS_TILE(256, false); break;
      case 512: ZK_FS_TILE(512, false); break;
      case 1024: ZK_FS_TILE(1024, false); break;
      default: ZK_FS_TILE(2048, false); break;
    }
  }
#undef ZK_FS_TILE
  ZK_LAUNCH_CHECK();
  fs_check<<<(unsigned)((tiles + FK_T - 1) / FK_T), FK_T, 0, st>>>(
      n_dev, n_cap, rent, rexit, rmeta, base, bsum, mins, grid + FL_NB, blist);
  ZK_LAUNCH_CHECK();
  fs_link<<<fl_blocks(), FL_T, 0, st>>>(buf, n_dev, n_cap, maxp, sx, list, rcnt,
                                 pre, rent, rexit, rmeta, base, cap, result,
                                 lbw + 2 * tiles, blist, bsum, mins, lastk,
                                 grid, lbw, cx, dbg ? dbg + 8 * tiles : nullptr);
  ZK_LAUNCH_CHECK();
  fs_rows<<<(unsigned)((tiles + 3) / 4), 256, 0, st>>>(
      buf, n_dev, n_cap, list, pre, rmeta, rent, rexit, base, bsum, lastk,
      foff, flen, cap, lbw);
  ZK_LAUNCH_CHECK();
  return 0;
}

int zk_frame_scan4(const uint8_t* buf, const int64_t* n_dev, int64_t n_cap,
                   int64_t maxp, uint8_t* ws, int64_t ws_bytes, int64_t* foff,
                   int32_t* flen, int64_t cap, int64_t* result, int32_t window,
                   int32_t clean, hipStream_t st) {
  return zk_frame_scan5(buf, n_dev, n_cap, maxp, ws, ws_bytes, foff, flen,
                        cap, result, window, clean, 0, st);
}

int zk_frame_scan3(const uint8_t* buf, const int64_t* n_dev, int64_t n_cap,
                   int64_t maxp, uint8_t* ws, int64_t ws_bytes, int64_t* foff,
                   int32_t* flen, int64_t cap, int64_t* result, int32_t window,
                   hipStream_t st) {
  return zk_frame_scan4(buf, n_dev, n_cap, maxp, ws, ws_bytes, foff, flen, cap,
                        result, window, 0, st);
}

// Chain statistics of the last scan of workspace `ws` over a buffer of
// n_cap bytes, into out3 (host): tiles without a speculated entry, tiles
// re-walked, repair rounds.
// out4: tiles without a speculated entry, tiles re-walked, repair rounds,
// tiles a chase looked up
int zk_frame_scan_stats(const uint8_t* ws, int64_t n_cap, int32_t window,
                        uint32_t* out4, hipStream_t st) {
  using namespace zk;
  (void)window;
  FsPlan p = fs_plan(n_cap);
  const uint64_t* lbw = (const uint64_t*)(ws + p.off_lbw);
  for (int k = 0; k < 4; ++k)
    if (hipMemcpyAsync(out4 + k, lbw + 2 * p.tiles + (k + 1) % 4, 4,
                       hipMemcpyDeviceToHost, st) != hipSuccess)
      return -1;
  if (hipStreamSynchronize(st) != hipSuccess) return -1;
  // counters since the last read (scans of a clean workspace skip the
  // memset that used to reset them)
  if (hipMemsetAsync((void*)(lbw + 2 * p.tiles), 0, 4 * 8, st) !=
      hipSuccess)
    return -1;
  return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
}

// rows = tiles + 1: the last row is fs_link's phase clock of a chase repair
// (start, chases done, barrier, links checked, end; [6] / [7] the exact
// chase's start and end)
int zk_frame_scan_dbg(int64_t* host, int64_t tiles) {
  if (!zk::g_dbg || tiles > zk::g_dbg_tiles + 1) return -1;
  return hipMemcpy(host, zk::g_dbg, tiles * 8 * 8, hipMemcpyDeviceToHost) ==
                 hipSuccess ? 0 : -1;
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
                        result, 2048, st);
}

}  // extern "C"

// K1 — parallel length-prefixed frame scan.
//
// Reference: ZKDecodeStream._transform (lib/zk-streams.js:39-65) walks the
// i32-BE length chain one frame at a time and memmoves the remainder per
// packet (O(bytes x packets)).  The chain is inherently
// sequential; we make it parallel over 4 KiB tiles in three launches:
//
//  fs_tile   ONE WAVE per tile (or per group of G = 2 / 4 tiles on streams
//            of large frames), two waves a workgroup, no barriers.  The tile
//            is staged into the wave's LDS once; everything else runs there:
//            1. nodes: every position whose i32-BE word is a plausible
//               length (8 <= len < 4 KiB; any legal length inside the entry
//               window) is a node, found 64 positions a lane;
//            2. the chain map: each node's successor (p + 4 + len) is
//               resolved by POINTER JUMPING over the node table in
//               registers (log2(chain length) rounds, ~5-7 on GET streams),
//               so every node knows where its chain leaves the tile, how
//               many frames it takes and whether it dies (a garbage entry
//               lands on a non-node within a hop or two);
//            3. the tile's candidate entries for the next tile — the exits
//               of the chains rooted in the window — go out in ONE packed
//               64-bit word (ready bit + five 12-bit offsets, a relaxed
//               agent-scope store: no release fence, which costs an L2
//               writeback per wave on a multi-XCD part);
//            4. the entry: the tile before's candidates, each looked up in
//               the map (the first whose chain survives is the entry; every
//               candidate's exit goes to `cx`, the entry -> exit map the
//               repair chases through);
//            5. the entry's chain read out of the map into the tile's list
//               of frame starts (a chain the map left open — a short frame
//               on it — is walked serially, as is a join onto the preferred
//               chain).
//            A group maps its first tile and walks the chain on through the
//            others (one LDS hop a frame), then checks its entry in a
//            register table of the first tile's window roots.
//  fs_link   The check over a grid of 16 workgroups (one wave per 64 tiles:
//            is each tile's entry the exit of the tile before, the first
//            terminal, the in-block frame counts; a launch of its own until
//            round 4 — moving it into fs_tile cost the tiles' ends more than
//            the launch), then a ticket: the LAST block to finish its check
//            goes on alone, no block waits for another (no grid barrier, so
//            no co-residency is assumed).  No broken link before the first
//            terminal (the usual case): it scans the block totals into row
//            bases, done.  Otherwise the repair: a few broken links are
//            chased in parallel waves — from each, forward while the next
//            link stays broken, the exact entry of a tile looked up among
//            the candidates fs_tile mapped (`cx`), so a run of tiles costs a
//            few instructions each; many, or what the chases leave, by the
//            tail: exact chases from the leftmost broken link, tiles whose
//            entry is no candidate walked, tiles covered whole by one frame
//            filled in one step; then the counts are scanned up to the first
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
// fs_link threads (512: 256 VGPRs a lane — with 1024 the chase and the walk
// inlined together spilled to scratch, 0.64 us a looked-up tile)
constexpr int FL_T = 512;
constexpr int FL_U = 8;                    // fs_link loads per batch
// fs_link's grid words (see fl_check's caller)
constexpr int FL_NB = 2;                   // broken links the check saw
constexpr int FL_GW = FL_NB + 1;
constexpr int FL_LOC = 1024;               // a block's own broken links
constexpr int FL_BROUNDS = 8;             // the last block's repair rounds
constexpr int FL_DBG_BLOCKS = 16;          // fs_link blocks with a debug clock
constexpr int FL_DBG_ROWS = 6;             // fs_link's debug rows past the tiles
// A block's own round over the broken links it found, before its ticket:
// off (the threshold is past any count).  Measured with the threshold at 64
// (tools/microbench/fl_probe.py, profiles/r5_fs_link_ab.md): the phantom-chain
// stream 0.69 ms a scan (one block walked 82 tiles serially before the last
// block could chase the region), 0.27 ms without; the dense and no-spec
// streams the same either way.
constexpr int FL_LOCAL_MIN = 1 << 30;
// The last block's one exact chase before its rounds (many broken links):
// tiles it may walk before it leaves the rest to the rounds
constexpr uint32_t FL_CHASE_WALKS = 16;
// Count blocks: frame counts scanned per FK_T tiles (one wave's worth)
constexpr int FK_T = 64;
// The workspace's words after the X flags (uint64, lbw + 2 * tiles): [0..3]
// stats, [4..5] the check's minima, [6] the last live tile, [7] this scan's
// tiles without a speculated entry (fs_tile counts, fs_rows clears),
// [8, 8 + FL_GW) fs_link's grid words, [16, 32) its barrier words (the big
// repair, see fs_link)
constexpr int LW_MINS = 4, LW_LAST = 6, LW_NOSPEC = 7, LW_GRID = 8;
constexpr int LW_BIG = 16;
constexpr int LW_END = 32;
static_assert(LW_GRID + FL_GW <= LW_BIG, "grid words");
// The big repair (barrier rounds over the grid) when a scan has more tiles
// without a speculated entry than this
constexpr unsigned FL_BIG_NOSPEC = 256;
constexpr int FL_GROUNDS = 6;              // its grid rounds
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

// ---- per-tile records shared with fs_link / fs_rows ------------------------
constexpr int FT_BITS = FT_S / 32;         // uint32 words per position map
constexpr int FT_XW = 2048 / 32;           // exit candidates: the next tile's
                                           // window positions (W <= 2048)

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

// The chain from tile-relative candidate entry e, walked in LDS (wave-
// uniform): does it survive this tile, and where does it leave it?
// Returns the absolute exit (>= the tile end) when it leaves the tile, or
// meets the survivor's path and the survivor leaves (its exit `send`),
// packed with the number of frames the chain starts in this tile
// (cx_exit / cx_cnt); FC_DEAD when it hits a bad length or meets a
// survivor that ends on one; FC_LIVE when it survives without a known exit
// (it reaches the stream end, or meets a survivor that ends there).
// fs_link's chase takes these as the tile's entry -> (exit, count) map.
// (fs_tile answers most candidates from its chain map; this exact walk is
// the fallback for chains the map leaves open.)
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

// ---- fs_tile: the tile's chain map, by pointer jumping ---------------------
//
// Every position p of the tile whose length word reads as a plausible frame
// body (minb <= len <= W - 4, the window covering the stream's frames;
// < FT_LIMIT in long-frame mode; in the entry window also any length up to
// maxp) is a NODE.  A node's successor is the next frame start, p + 4 + len:
// another node, or a ROOT where the chain ends inside the tile's view —
//   EXIT   the chain leaves the tile (val = its last frame's start: the exit
//          is that frame's end, read from the staged bytes);
//   END    the stream ends exactly at the last frame's end (val = its start);
//   PART   a frame (val) is cut by the stream end (its header or body);
//   BAD    a frame (val) has a length < 0 or > maxp (BAD_LENGTH);
//   SHORT  a frame (val) has a legal length below minb: the map does not
//          follow it (an exact serial walk does, when the chain matters).
// Pointer jumping (each round: node -> successor's successor, counts
// added) takes every node to its root in log2(frames per tile) rounds, all
// lanes busy: ~5 rounds on 192-byte frames, ~7 on 42-byte ones, where the
// round-3 kernel walked ~20 / ~90 dependent LDS hops on one lane after a
// merging frontier.  Lane l holds nodes l, l + 64, ... in registers (their
// positions and words), and every phase issues all of its LDS reads before
// it waits.  The map then answers, in O(1) each, what the tile chain logic
// needs: the exits of the window entries (the next tile's candidate
// entries), the survival / exit / frame count of the tile before's
// candidates (fs_link's candidate exit map), and the frame starts of the
// chosen entry's chain (slot index = count - the node's count to the root;
// a side branch landing on the chain is caught by the successor check and
// sent to the serial walk).  What fs_link / fs_rows read is
// unchanged: entry, exit, count, frame-start lists and candidate exits.
constexpr int FT_NMAX = 512;               // nodes a tile's map holds (GET
                                           // streams: 240-340; more: the
                                           // serial walks)
constexpr int FT_SLOTS = 352;              // chain slots (frames >= 12 bytes)
constexpr int32_t FT_LIMIT = FT_S;         // node lengths below this
enum : uint32_t {
  RK_NODE = 0, RK_EXIT = 1, RK_END = 2, RK_PART = 3, RK_BAD = 4, RK_SHORT = 5
};
// node word: kind (3 bits) | val (13 bits: successor node or a position) |
// frame starts from the node to the root (16 bits)
ZK_DEV uint32_t rk(uint32_t kind, uint32_t val, uint32_t cnt) {
  return kind << 29 | val << 16 | cnt;
}
ZK_DEV uint32_t rk_kind(uint32_t w) { return w >> 29; }
ZK_DEV uint32_t rk_val(uint32_t w) { return (w >> 16) & 0x1FFF; }
ZK_DEV uint32_t rk_cnt(uint32_t w) { return w & 0xFFFF; }

// LDS layout per wave (7.6 KiB: 20 waves a CU): staged tile | node masks
// of the 64 position blocks | nodes before each block | node words | R:
// node positions while the map is built, then the chain slots (or the
// serial walks' survivor bits) and the exit candidate bits
constexpr int FT_SLOT_B = 704;             // >= FT_SLOTS * 2, >= FT_BITS * 4
constexpr int FT_O_BLK = FT_STAGE;         // uint64 [64]
constexpr int FT_O_BASE = FT_O_BLK + 64 * 8;   // uint16 [64]
constexpr int FT_O_PK = FT_O_BASE + 64 * 2;
constexpr int FT_O_R = FT_O_PK + FT_NMAX * 4;
constexpr int FT_R_B = FT_NMAX * 2 > FT_SLOT_B + FT_XW * 4
                           ? FT_NMAX * 2 : FT_SLOT_B + FT_XW * 4;
constexpr int FT_O_XB = FT_O_R + FT_SLOT_B;
constexpr int FT_LDS = FT_O_R + FT_R_B;
static_assert(FT_SLOT_B >= FT_SLOTS * 2 && FT_SLOT_B >= FT_BITS * 4, "slots");
static_assert(FT_STAGE % 16 == 0 && FT_LDS % 16 == 0, "LDS alignment");

// Big-endian i32 at byte p from the two aligned dwords around it.
ZK_DEV int32_t be32_of(uint32_t lo, uint32_t hi, int32_t p) {
  return (int32_t)bswap32(__builtin_amdgcn_alignbyte(hi, lo, p & 3));
}

// The node map of a tile: a mask of nodes per 64-position block and the
// nodes before each block (node indices follow positions).
struct FtBlk {
  const uint64_t* mask;
  const uint16_t* base;
};

// Is tile position q (< FT_S) a node; its index if so.
ZK_DEV bool ft_node(const FtBlk& blk, int32_t q, int32_t& idx) {
  const uint64_t m = blk.mask[q >> 6];
  const int32_t b = blk.base[q >> 6];
  const uint64_t bit = 1ull << (q & 63);
  idx = b + __popcll(m & (bit - 1));
  return (m & bit) != 0;
}

// The root word of a chain continuing at NON-node position q (< FT_S) whose
// length word reads len, after `before` frame starts.
ZK_DEV uint32_t ft_classify(int32_t q, int32_t len, int32_t nrel,
                            int32_t maxp, int32_t minb, uint32_t before) {
  if (q + 4 > nrel) return rk(RK_PART, q, before);
  if ((uint32_t)len > (uint32_t)maxp) return rk(RK_BAD, q, before);
  const int32_t nx = q + 4 + len;
  if (nx > nrel) return rk(RK_PART, q, before);
  if (len < minb) return rk(RK_SHORT, q, before);
  // a legal length >= FT_LIMIT (not a node): the frame leaves the tile
  if (nx >= FT_S) return rk(RK_EXIT, q, before + 1);
  return nx == nrel ? rk(RK_END, q, before + 1) : rk(RK_SHORT, q, before);
}

// Root word of the chain entering at tile position e (wave-uniform; e <
// nrel, the map built).
ZK_DEV uint32_t ft_root_at(const uint8_t* sb, const FtBlk& blk,
                           const uint32_t* pk, int32_t e, int32_t nrel,
                           int32_t maxp, int32_t minb) {
  int32_t j;
  if (ft_node(blk, e, j)) return pk[j];
  return ft_classify(e, lds_be32(sb, e), nrel, maxp, minb, 0);
}

// End of the frame starting at tile position p (its length word staged).
ZK_DEV int32_t ft_next(const uint8_t* sb, int32_t p) {
  return p + 4 + lds_be32(sb, p);
}

// The candidate-exit value (ft_cand's) of a chain with root word w.
ZK_DEV int64_t ft_cx(const uint8_t* sb, uint32_t w, int64_t ts) {
  switch (rk_kind(w)) {
    case RK_EXIT:
      return (ts + ft_next(sb, (int32_t)rk_val(w))) |
             ((int64_t)rk_cnt(w) << CX_SHIFT);
    case RK_BAD: return FC_DEAD;
    default: return FC_LIVE;                 // END / PART
  }
}

// The survivor end code (sx) of a chain with root word w.
ZK_DEV int64_t ft_send(const uint8_t* sb, uint32_t w, int64_t ts) {
  const int32_t v = (int32_t)rk_val(w);
  switch (rk_kind(w)) {
    case RK_EXIT: return ts + ft_next(sb, v);
    case RK_END: return TERM | (ts + ft_next(sb, v));
    case RK_BAD: return TERM | TBAD | (ts + v);
    default: return TERM | (ts + v);         // PART
  }
}

// This lane's nodes i = lane + 64 k: positions (-1: none) and words.
template <int NK>
struct FtNodes {
  int32_t p[NK];
  uint32_t w[NK];
};

// Successors of this lane's nodes, then pointer jumping until every node's
// word is its root's (kind, val) with the frame count from it.  Returns the
// jumping rounds.
template <int NK>
ZK_DEV int ft_build(FtNodes<NK>& me, const uint8_t* sb, const FtBlk& blk,
                    uint32_t* pk, const uint16_t* pos, int32_t N,
                    int32_t nrel, int32_t maxp, int32_t minb, int lane) {
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int32_t i = lane + 64 * k;
    const int32_t p = pos[i < N ? i : 0];
    me.p[k] = i < N ? p : -1;
  }
  uint32_t a[NK], b[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int32_t q = me.p[k] < 0 ? 0 : me.p[k] & ~3;
    a[k] = *(const uint32_t*)(sb + q);
    b[k] = *(const uint32_t*)(sb + q + 4);
  }
  int32_t nx[NK];
  uint64_t bm[NK];
  uint32_t bb[NK], c[NK], d[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int32_t p = me.p[k] < 0 ? 0 : me.p[k];
    nx[k] = p + 4 + be32_of(a[k], b[k], p);
    const int32_t q = nx[k] < FT_S ? nx[k] : 0;
    bm[k] = blk.mask[q >> 6];
    bb[k] = blk.base[q >> 6];
    c[k] = *(const uint32_t*)(sb + (q & ~3));
    d[k] = *(const uint32_t*)(sb + (q & ~3) + 4);
  }
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int32_t p = me.p[k];
    const int32_t q = nx[k];
    uint32_t r;
    if (q > nrel) {
      r = rk(RK_PART, p, 0);
    } else if (q >= FT_S) {
      r = rk(RK_EXIT, p, 1);
    } else if (q == nrel) {
      r = rk(RK_END, p, 1);
    } else {
      const uint64_t bit = 1ull << (q & 63);
      if (bm[k] & bit)
        r = rk(RK_NODE, bb[k] + __popcll(bm[k] & (bit - 1)), 1);
      else
        r = ft_classify(q, be32_of(c[k], d[k], q), nrel, maxp, minb, 1);
    }
    me.w[k] = r;
    if (p >= 0) pk[lane + 64 * k] = r;
  }
  __builtin_amdgcn_wave_barrier();
  int rounds = 0;
  for (;;) {
    uint32_t q[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const bool go = me.p[k] >= 0 && rk_kind(me.w[k]) == RK_NODE;
      q[k] = pk[go ? rk_val(me.w[k]) : 0];
    }
    bool more = false;
    uint32_t nw[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      nw[k] = me.w[k];
      if (me.p[k] >= 0 && rk_kind(me.w[k]) == RK_NODE) {
        nw[k] = (q[k] & 0xFFFF0000u) | (rk_cnt(me.w[k]) + rk_cnt(q[k]));
        more |= rk_kind(q[k]) == RK_NODE;
      }
    }
    // every read of the round is issued before its first write (the
    // wave's LDS operations complete in order)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      if (nw[k] != me.w[k]) pk[lane + 64 * k] = nw[k];
      me.w[k] = nw[k];
    }
    __builtin_amdgcn_wave_barrier();
    ++rounds;
    if (!__ballot(more)) break;
  }
  return rounds;
}

// The window entries' exits into xbits (this tile's candidate entries of
// the next one) and the preferred chain: the window entry with the longest
// chain, else (LONG) the first node whose chain leaves the tile.  Returns
// its position (-1: none) and its exit past the tile end in `sx`.
template <int W, bool LONG, int NK>
ZK_DEV int32_t ft_cands(const FtNodes<NK>& me, const uint8_t* sb,
                        uint32_t* xbits, int32_t& sx) {
  uint32_t a[NK], b[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const bool ex = rk_kind(me.w[k]) == RK_EXIT && me.p[k] >= 0 &&
                    (LONG || me.p[k] < W);
    const int32_t v = ex ? (int32_t)rk_val(me.w[k]) : 0;
    a[k] = *(const uint32_t*)(sb + (v & ~3));
    b[k] = *(const uint32_t*)(sb + (v & ~3) + 4);
  }
  // keys: (count, -position) above the exit, so the max carries its exit
  uint64_t best = 0, first = 0;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int32_t p = me.p[k];
    if (p < 0 || rk_kind(me.w[k]) != RK_EXIT || (!LONG && p >= W)) continue;
    const int32_t v = (int32_t)rk_val(me.w[k]);
    const uint32_t x = (uint32_t)(v + 4 + be32_of(a[k], b[k], v) - FT_S);
    if (p < W) {
      if (x < (uint32_t)W)
        __hip_atomic_fetch_or(&xbits[x >> 5], 1u << (x & 31),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      const uint64_t key = (uint64_t)(rk_cnt(me.w[k]) << 16 |
                                      (uint32_t)(0xFFFF - p)) << 32 | x;
      best = best > key ? best : key;
    } else if (LONG) {
      const uint64_t key = (uint64_t)(0xFFFF - p) << 32 | x;
      first = first > key ? first : key;
    }
  }
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    const uint64_t o = (uint64_t)__shfl_xor((long long)best, s, 64);
    best = best > o ? best : o;
    if (LONG) {
      const uint64_t f = (uint64_t)__shfl_xor((long long)first, s, 64);
      first = first > f ? first : f;
    }
  }
  const uint64_t k = best ? best : (LONG ? first : 0);
  if (!k) return -1;
  sx = (int32_t)(uint32_t)k;
  return 0xFFFF - (int32_t)((k >> 32) & 0xFFFF);
}

// ft_cands for a tile without a map (more than FT_NMAX nodes: payloads of
// small big-endian words, each a plausible length).  The window's first
// 128 nodes are walked, one chain per lane and round, all lanes at once
// (per-lane LDS hops); their exits and the preferred chain are chosen as
// ft_cands chooses them.  Without this the tile published no candidate,
// the next one had no speculated entry, and a run of such tiles became a
// serial repair.
template <int W>
ZK_DEV int32_t ft_cands_walk(const uint8_t* sb, const FtBlk& blk,
                             uint32_t* xbits, int32_t nrel, int32_t maxp,
                             int32_t& sx, int lane) {
  uint64_t best = 0;
  for (int r = 0; r < 2; ++r) {
    // this lane's window node: index lane + 64 r in position order
    int32_t want = lane + 64 * r, p = -1;
    for (int b = 0; b < W / 64 && p < 0; ++b) {
      uint64_t m = blk.mask[b];
      const int32_t c = __popcll(m);
      if (want < c) {
        for (int k = 0; k < want; ++k) m &= m - 1;
        p = b * 64 + (int32_t)__builtin_ctzll(m);
      } else {
        want -= c;
      }
    }
    if (!__ballot(p >= 0)) break;
    int32_t c = p, cnt = 0, x = -1;
    bool live = p >= 0;
    while (live) {
      if (c + 4 > nrel) break;
      const int32_t len = lds_be32(sb, c);
      if ((uint32_t)len > (uint32_t)maxp) break;
      const int32_t nx = c + 4 + len;
      if (nx > nrel) break;
      ++cnt;
      if (nx >= FT_S) { x = nx - FT_S; break; }
      c = nx;
    }
    if (x >= 0) {
      if (x < W)
        __hip_atomic_fetch_or(&xbits[x >> 5], 1u << (x & 31),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      const uint64_t key = (uint64_t)((uint32_t)cnt << 16 |
                                      (uint32_t)(0xFFFF - p)) << 32 |
                           (uint32_t)x;
      best = best > key ? best : key;
    }
  }
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    const uint64_t o = (uint64_t)__shfl_xor((long long)best, s, 64);
    best = best > o ? best : o;
  }
  if (!best) return -1;
  sx = (int32_t)(uint32_t)best;
  return 0xFFFF - (int32_t)((best >> 32) & 0xFFFF);
}

// The frame starts of the chain entering at tile position e with root word
// w into the wave's slots (slot k = the k-th start): every node of that
// root with count c <= D at or after e lands in slot D - c; the successor
// check over the slots rejects a side branch sharing the root and count.
// Returns D, or -1 when the chain needs the exact serial walk.
template <int NK>
ZK_DEV int32_t ft_chain(const FtNodes<NK>& me, const uint8_t* sb,
                        const FtBlk& blk, uint16_t* slot, int32_t e,
                        uint32_t w, int lane) {
  const uint32_t kind = rk_kind(w);
  const int32_t D = (int32_t)rk_cnt(w);
  if (kind == RK_SHORT || kind == RK_BAD || D > FT_SLOTS) return -1;
  if (D == 0) return 0;
  const uint32_t root = w >> 16;
  int32_t hits = 0;
  bool on[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int32_t c = (int32_t)rk_cnt(me.w[k]);
    const int32_t p = me.p[k];
    on[k] = p >= e && (me.w[k] >> 16) == root && c >= 1 && c <= D;
    if (on[k]) slot[D - c] = (uint16_t)p;
    hits += __popcll(__ballot(on[k]));
  }
  __builtin_amdgcn_wave_barrier();
  // the chain's nodes: its D frame starts, less the last one when that
  // frame (a long one) is not a node
  int32_t want = D;
  if (lane == 0) {
    slot[0] = (uint16_t)e;
    if (kind == RK_EXIT || kind == RK_END) slot[D - 1] = (uint16_t)rk_val(w);
  }
  if (kind == RK_EXIT || kind == RK_END) {
    int32_t j;
    if (!ft_node(blk, (int32_t)rk_val(w), j)) --want;
  }
  __builtin_amdgcn_wave_barrier();
  // as many hits as chain nodes: no side branch shares the root and a
  // count, every slot holds the chain's start
  if (hits == want) return D;
  // the successor check: every slot's frame ends at the next slot
  auto linked = [&]() {
    bool ok = true;
    for (int32_t k = lane; k < D; k += 64) {
      const int32_t p = slot[k];
      const int32_t nx = ft_next(sb, p);
      if (k + 1 < D) {
        ok &= nx == (int32_t)slot[k + 1];
      } else if (kind == RK_PART) {
        ok &= nx == (int32_t)rk_val(w);
      }
    }
    return __ballot(!ok) == 0;
  };
  if (linked()) return D;
  // Side branches share the root and a count: a length-like word inside a
  // frame that ends where its frame does — a create reply's path length
  // (4 + len past it is the next frame's start: every storm reply frame) —
  // lands on the chain one frame on, and the slot may hold it.  The chain's
  // start is the first of them, so each slot keeps its smallest position
  // (a few rounds: lanes writing one slot at once leave any of their
  // values), and the successor check decides again.  Without it every storm
  // reply tile took the serial walk (24 us of its 77,
  // tools/microbench/k1_bench.py --workload storm).
  for (int it = 0; it < 8; ++it) {
    int32_t cur[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k)
      cur[k] = on[k] ? (int32_t)slot[D - (int32_t)rk_cnt(me.w[k])] : 0;
    bool wr = false;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      if (on[k] && me.p[k] < cur[k]) {
        slot[D - (int32_t)rk_cnt(me.w[k])] = (uint16_t)me.p[k];
        wr = true;
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (!__ballot(wr)) break;
  }
  return linked() ? D : -1;
}

ZK_DEV int64_t ft_walk(const uint8_t* sb, int32_t c, int32_t nrel,
                       int32_t maxp32, int64_t ts, uint16_t* L, int32_t& mo,
                       int lane);

// What fs_tile's steps 2-5 need from the kernel.
struct FtCtx {
  const uint8_t* buf;
  uint16_t* list;
  uint16_t* pre;
  int64_t* sx;
  uint64_t* lbw;
  int64_t* rec_entry;
  int64_t* rec_exit;
  int64_t* rec_meta;
  int32_t* rcount;
  int64_t* dbg;
  int64_t* cx;
  uint64_t* stats;
  uint8_t* sb;
  FtBlk blk;
  uint32_t* pk;
  uint16_t* pos;
  uint16_t* slot;
  uint32_t* sbits;
  uint32_t* xbits;
  int64_t n, t, ts, tend, t_0, t_s, t_d;
  int32_t nrel, maxp32, minb, N, misspec;
  bool nospec;
  int lane;
};

template <int W, bool LONG, int NK>
ZK_DEV int64_t fs_tile_rest(const FtCtx& cx_, bool mapped) {
  const FtCtx& C = cx_;
  const int lane = C.lane;
  const uint8_t* sb = C.sb;
  const int64_t n = C.n, t = C.t, ts = C.ts, tend = C.tend;
  const int32_t nrel = C.nrel, maxp32 = C.maxp32, minb = C.minb;
  constexpr int XW = W / 32;                // candidate words used
  FtNodes<NK> me;
  int rounds = 0;
  if (mapped)
    rounds = ft_build<NK>(me, sb, C.blk, C.pk, C.pos, C.N, nrel, maxp32, minb,
                          lane);
  // the positions are in registers now: R becomes the slots / bits
  for (int k = lane; k < FT_R_B / 4; k += 64) C.sbits[k] = 0u;
  __builtin_amdgcn_wave_barrier();
  const int64_t t_f = C.dbg ? wall_clock64() : 0;

  // ---- 3. the window entries' exits: this tile's candidates for the next -
  int32_t px = -1, sp = -1;
  {
    int32_t x = -1;
    sp = mapped ? ft_cands<W, LONG, NK>(me, sb, C.xbits, x)
                : ft_cands_walk<W>(sb, C.blk, C.xbits, nrel, maxp32, x, lane);
    if (sp >= 0 && x >= 0 && x < (LONG ? FT_S - 1 : W)) px = x;
  }
  // Candidates go out packed in ONE 64-bit word (a relaxed agent-scope
  // store: no fence, no L2 write-back on this multi-XCD part): bit 63 =
  // ready, five 12-bit slots of offset + 1 (0 = empty), slot 0 the preferred
  // one, then up to four other in-window exits in offset order.
  __builtin_amdgcn_wave_barrier();
  uint64_t word = (uint64_t)1 << 63;
  if (px >= 0) word |= (uint64_t)(px + 1);
  {
    uint32_t xw = lane < XW ? C.xbits[lane] : 0u;
    if (px >= 0 && px < W && lane == (px >> 5)) xw &= ~(1u << (px & 31));
    uint64_t any = __ballot(xw != 0);
    int nsl = 1;
    if (px < 0 && any) {
      // no preferred exit: the first in-window one
      const int wl = (int)__builtin_ctzll(any);
      const uint32_t bits = (uint32_t)__builtin_amdgcn_readlane((int)xw, wl);
      const int x0 = wl * 32 + (int)__builtin_ctz(bits);
      word |= (uint64_t)(x0 + 1);
      if (lane == wl) xw &= ~(1u << (x0 & 31));
      any = __ballot(xw != 0);
    }
    while (any && nsl < 5) {
      const int wl = (int)__builtin_ctzll(any);
      uint32_t bits = (uint32_t)__builtin_amdgcn_readlane((int)xw, wl);
      while (bits && nsl < 5) {
        const int bit = (int)__builtin_ctz(bits);
        bits &= bits - 1;
        word |= (uint64_t)(wl * 32 + bit + 1) << (12 * nsl);
        ++nsl;
      }
      any &= any - 1;
    }
  }
  if (lane == 0) lb_store(&C.lbw[2 * t], word);    // 0 = not yet
  const int64_t t_1 = C.dbg ? wall_clock64() : 0;

  // ---- 4. the entry: the tile before's candidates, checked in the map ----
  int64_t E = 0;
  bool none = false;
  uint32_t wE = 0;               // the entry's root word, when wE_ok
  bool wE_ok = false;
  if (t > 0 && C.nospec) {
    // (tests: every tile but the first without a speculated entry, the
    // worst case of the link repair; no candidate exits either)
    none = true;
    if (lane < 5) C.cx[5 * t + lane] = FC_DEAD;
  } else if (t > 0) {
    // Tile t-1 is running or done.  Poll with exponential back-off: these
    // loads bypass the caches, and thousands of waves polling every few
    // hundred cycles flood the fabric.
    uint64_t x;
    int nap = 0;
    const uint64_t t_w = wall_clock64();
    for (;;) {
      x = lb_load(&C.lbw[2 * (t - 1)]);
      if (x != 0) break;
      if (wall_clock64() - t_w > FT_WAIT_TICKS) break;   // no speculation
      // the tile before usually publishes within a microsecond: short
      // naps first (128 cycles), then back off
      if (nap < 16) __builtin_amdgcn_s_sleep(2);
      else if (nap < 32) __builtin_amdgcn_s_sleep(8);
      else __builtin_amdgcn_s_sleep(32);
      ++nap;
    }
    // The first candidate whose chain survives this tile is the entry (a
    // garbage exit of the tile before dies on a bad length here).  Every
    // candidate's outcome goes to `cx`: where two chains both survive tile
    // after tile (a phantom chain), fs_link's chase follows the exact one
    // through this map instead of re-walking every tile.  Lane s checks
    // candidate s in the map; chains the map leaves open are walked.
    const int32_t v = lane < 5 ? (int32_t)((x >> (12 * lane)) & 0xFFF) : 0;
    const bool has = v != 0 && ts + (v - 1) < n;
    const int32_t e = v - 1;
    uint32_t we = 0;
    if (has && mapped) we = ft_root_at(sb, C.blk, C.pk, e, nrel, maxp32, minb);
    const bool open = has && (!mapped || rk_kind(we) == RK_SHORT);
    int64_t xe = has && !open ? ft_cx(sb, we, ts) : FC_DEAD;
    for (uint64_t um = __ballot(open); um; um &= um - 1) {
      const int l = (int)__builtin_ctzll(um);
      const int32_t el = __builtin_amdgcn_readlane(e, l);
      const int64_t r = ft_cand(sb, C.sbits, el, nrel, maxp32, -1, n, ts, 0,
                                lane);
      if (lane == l) xe = r;
    }
    if (lane < 5) C.cx[5 * t + lane] = xe;
    const uint64_t hm = __ballot(has);
    const uint64_t lm = __ballot(has && xe != FC_DEAD);
    int64_t first = -1;
    E = -1;
    if (lm) {
      const int l = (int)__builtin_ctzll(lm);
      E = ts + __builtin_amdgcn_readlane(e, l);
      wE = (uint32_t)__builtin_amdgcn_readlane((int)we, l);
      wE_ok = mapped && !__builtin_amdgcn_readlane((int)open, l);
    }
    if (hm) first = ts + __builtin_amdgcn_readlane(e, (int)__builtin_ctzll(hm));
    if (E < 0) E = first;        // no live candidate: the first one
    // (tests: every misspec-th tile takes a garbage entry one byte past the
    // chosen one, the link repair's adversary)
    if (C.misspec > 0 && t % C.misspec == 1 && E >= 0 && E + 1 < n) {
      ++E;
      wE_ok = false;
    }
    none = E < 0;
  }
  const int64_t t_2 = C.dbg ? wall_clock64() : 0;

  // ---- 5. the chain's frame starts ---------------------------------------
  // The entry's chain when the map has it (the usual case: its starts are
  // the tile's list, no walk); otherwise the preferred chain's starts are
  // the survivor list (fs_link's repair joins it) and the entry is walked
  // serially until it joins it, dies or leaves, as round 3 did.
  uint16_t* L = C.list + t * FT_LMAX;
  FcWalk wk{E, 0, 0, -1, false, false};
  int64_t send = -1;
  int32_t m = 0;
  bool done = false;
  const int32_t erel = (int32_t)(E - ts);
  if (!none && erel >= nrel) {
    // the entry is the stream's end
    send = TERM | E;
    fc_join_end(wk, send, n);
    done = true;
  } else if (!none && mapped) {
    const uint32_t we = wE_ok ? wE
                              : ft_root_at(sb, C.blk, C.pk, erel, nrel, maxp32,
                                           minb);
    const int32_t D = ft_chain<NK>(me, sb, C.blk, C.slot, erel, we, lane);
    if (D >= 0) {
      for (int32_t k = lane; k < D; k += 64) L[k] = C.slot[k];
      m = D;
      send = ft_send(sb, we, ts);
      wk.cnt = D;
      wk.js = D > 0 ? 0 : -1;
      fc_join_end(wk, send, n);
      done = true;
    }
  }
  if (!done) {
    // survivor list: the preferred chain's starts (from the map, or
    // walked when the tile has none)
    if (sp >= 0 && mapped) {
      const uint32_t ws = ft_root_at(sb, C.blk, C.pk, sp, nrel, maxp32, minb);
      const int32_t D = ft_chain<NK>(me, sb, C.blk, C.slot, sp, ws, lane);
      if (D > 0) {
        for (int32_t k = lane; k < D; k += 64) L[k] = C.slot[k];
        m = D;
        send = ft_send(sb, ws, ts);
      }
    } else if (sp >= 0) {
      __builtin_amdgcn_wave_barrier();
      send = ft_walk(sb, sp, nrel, maxp32, ts, L, m, lane);
      if (m == 0) send = -1;
    }
    __builtin_amdgcn_wave_barrier();
    // survivor bits from the list just stored (each lane rereads only what
    // it wrote itself)
    for (int k = lane; k < FT_SLOT_B / 4; k += 64) C.sbits[k] = 0u;
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < m; i += 64) {
      const int32_t q = L[i];
      __hip_atomic_fetch_or(&C.sbits[q >> 5], 1u << (q & 31),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    __builtin_amdgcn_wave_barrier();
    if (!none) {
      // join: walk from the entry until the survivor's path
      int64_t c = E;
      uint16_t* P = C.pre + t * FT_LMAX;
      int32_t np = 0;
      uint32_t ent = 0;
      for (;;) {
        if (c >= tend) { wk.exit = c; break; }
        if (c >= n) { wk.exit = n; break; }  // the stream ends cleanly
        const int32_t crel = (int32_t)(c - ts);
        const uint32_t smw = C.sbits[crel >> 5];
        const int32_t lraw = lds_be32(sb, crel);
        if ((smw >> (crel & 31)) & 1u) {
          // joined: the rest is the survivor's list from this start on
          static_assert(FT_BITS == 2 * 64, "two map words per lane");
          const int32_t cw = crel >> 5;
          int32_t s = 0;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int32_t wi = lane + 64 * h;
            const uint32_t wd = C.sbits[wi];
            s += wi < cw ? __popc(wd)
                         : (wi == cw ? __popc(wd & ((1u << (crel & 31)) - 1u))
                                     : 0);
          }
#pragma unroll
          for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
          wk.js = s;
          break;
        }
        const int32_t len = __builtin_amdgcn_readfirstlane(lraw);
        const int32_t nx = crel + 4 + len;
        if ((uint32_t)len > (uint32_t)maxp32 || nx > nrel) {
          wk.exit = c;
          wk.term = true;
          wk.bad = (crel + 4 <= nrel) && ((len < 0) | (len > maxp32));
          break;
        }
        ft_record(P, np, ent, crel, lane);
        c = ts + nx;
      }
      if (lane < (np & 63)) P[(np & ~63) + lane] = (uint16_t)ent;
      wk.np = np;
      wk.cnt = np;
      if (wk.js >= 0) {
        wk.cnt = np + (m - wk.js);
        fc_join_end(wk, send, n);
      }
    } else {
      // no speculated entry: the exit recorded is the survivor's (the
      // likely one), so fs_link's grid repair of the NEXT tile can start
      // from it in the same round as this tile's own repair
      if (m > 0) fc_join_end(wk, send, n);
      if (lane == 0) fc_stat(C.stats, 1, 1), fc_stat(C.stats, LW_NOSPEC, 1);
    }
  }
  if (lane == 0) {
    C.sx[t] = send;
    C.rcount[t] = m;
    C.rec_entry[t] = none ? -1 : E;
    C.rec_exit[t] = wk.exit;
    C.rec_meta[t] = fc_meta(wk);
    if (C.dbg) {
      int64_t* d = C.dbg + 8 * t;
      d[0] = C.t_0;
      d[1] = t_1;
      d[2] = t_2;
      d[3] = wall_clock64();
      d[4] = C.t_d;
      d[5] = (int64_t)C.N | (int64_t)rounds << 16 | (int64_t)done << 24;
      d[6] = C.t_s;
      d[7] = t_f;
    }
  }
  return send;
}

// ---- tile groups: the map once, then the chain walked on ------------------
// A group of G consecutive tiles is one wave's work (G > 1: streams whose
// frames are large, so a tile holds few of them).  The group's first tile
// gets the chain map as above; its preferred chain is then WALKED through
// the group's other tiles (staged one after the other into the same LDS;
// the next tile's bytes ride in registers while the walk runs), one
// dependent LDS hop per frame: ~20 hops a tile on 192-byte frames, where a
// map costs ~6 us of detection and jumping.  Only the group's first tile
// speculates an entry; the others' entries are the walk's exits, recorded
// as their only candidate (word + cx) so fs_link's chase sees the usual
// maps.  After its walk the group publishes its last exit and takes the
// group before's: the first tile's candidates are checked in a register
// table of its window positions' roots, kept from the map.

// Stage the 4 KiB tile at ts in registers (zero past n) / into LDS.
struct FtTileRegs {
  uint4 v[FT_S / 16 / 64];
  uint4 pad;
};
ZK_DEV void ft_load(const uint8_t* __restrict__ buf, int64_t n, int64_t ts,
                    int lane, FtTileRegs& r) {
  constexpr int PER = FT_S / 16 / 64;
  r.pad = make_uint4(0, 0, 0, 0);
  if (ts + FT_STAGE <= n) {
#pragma unroll
    for (int j = 0; j < PER; ++j)
      __builtin_memcpy(&r.v[j], buf + ts + 16 * (lane + 64 * j), 16);
    if (lane == 0) __builtin_memcpy(&r.pad, buf + ts + FT_S, 16);
  } else {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      uint8_t* b = (uint8_t*)&r.v[j];
      const int64_t g = ts + 16 * (lane + 64 * j);
      for (int k = 0; k < 16; ++k) b[k] = g + k < n ? buf[g + k] : 0;
    }
    if (lane == 0) {
      uint8_t* b = (uint8_t*)&r.pad;
      for (int k = 0; k < 16; ++k)
        b[k] = ts + FT_S + k < n ? buf[ts + FT_S + k] : 0;
    }
  }
}
ZK_DEV void ft_store(uint8_t* sb, const FtTileRegs& r, int lane) {
  constexpr int PER = FT_S / 16 / 64;
#pragma unroll
  for (int j = 0; j < PER; ++j) *(uint4*)(sb + 16 * (lane + 64 * j)) = r.v[j];
  if (lane == 0) *(uint4*)(sb + FT_S) = r.pad;
  __builtin_amdgcn_wave_barrier();
}

// The chain from tile-relative c through the staged tile (wave-uniform),
// its frame starts into L; returns the end code (sx) and the count.
// After two frames of one size, a hop reads besides the frame's length
// word (lane 0) the words where the next 63 frames start if they are of
// that size too (lane l: l frames on), so a run of equal frames — every GET
// reply of a 100-byte node is 192 bytes — is taken in one step: the
// leading lanes whose word repeats the length.  One LDS round trip a step
// either way (a group's walked tiles were ~20 dependent hops each, 34 us
// of a 47 us group, tools/microbench/k1_bench.py); streams of varied
// frames keep the one-address hop (a vector address on every hop cost the
// 0-200 B GET stream 3 %) and the records gathered 64 to a store.
ZK_DEV int64_t ft_walk(const uint8_t* sb, int32_t c, int32_t nrel,
                       int32_t maxp32, int64_t ts, uint16_t* L, int32_t& mo,
                       int lane) {
  int32_t m = 0, pb = 0;              // records [pb, m) pending in ent
  uint32_t ent = 0;
  int64_t send;
  // (the walk is wave-uniform: the position and the bounds in SGPRs)
  c = __builtin_amdgcn_readfirstlane(c);
  nrel = __builtin_amdgcn_readfirstlane(nrel);
  const int32_t lim = min((int32_t)FT_S, nrel);
  if (c >= nrel) {
    send = TERM | (ts + c);
  } else {
    int32_t len = 0, nx = 0, last = 0;      // last: the last frame's size
    bool ok = true, fin = false;
    while (!fin) {
      len = __builtin_amdgcn_readfirstlane(lds_be32(sb, c));
      nx = c + 4 + len;
      ok = (uint32_t)len <= (uint32_t)maxp32 && nx <= nrel;
      if (!ok) break;
      ent = lane == (m & 63) ? (uint32_t)c : ent;
      ++m;
      if ((m & 63) == 0) {
        const int32_t q = m - 64 + lane;
        if (q >= pb) L[q] = (uint16_t)ent;
        pb = m;
      }
      if (nx >= lim) break;
      c = nx;
      if (4 + len != last) {
        last = 4 + len;
        continue;
      }
      // two frames of one size: steps over the run (lane l reads where
      // frame l of it would start); frames 0 .. a-1 lie back to back with
      // that length, and the walk ends after the first reaching the tile's
      // end.  A step that takes none goes back to the hop above.
      const int32_t st = last;
      for (;;) {
        const int64_t s64 = (int64_t)c + (int64_t)lane * st;
        const int32_t sp = s64 < lim ? (int32_t)s64 : lim;
        const int32_t lv = sp < lim ? lds_be32(sb, sp) : -1;
        const bool acc = sp < lim && lv == st - 4 && sp + st <= nrel;
        const uint64_t no = ~__ballot(acc);
        const int32_t a = no ? (int32_t)__builtin_ctzll(no) : 64;
        if (a == 0) break;
        const uint64_t end = __ballot(acc && sp + st >= lim);
        const int32_t f = end ? (int32_t)__builtin_ctzll(end) : 64;
        const int32_t r = min(a, f + 1);
        const int32_t q = (m & ~63) + lane;
        if (q >= pb && q < m) L[q] = (uint16_t)ent;
        if (lane < r) L[m + lane] = (uint16_t)sp;
        m += r;
        pb = m;
        nx = c + r * st;
        len = st - 4;
        if (nx >= lim) {
          fin = true;
          break;
        }
        c = nx;
      }
    }
    if (!ok) {
      const bool bad = (c + 4 <= nrel) && ((len < 0) | (len > maxp32));
      send = TERM | (bad ? TBAD : 0) | (ts + c);
    } else if (nx >= FT_S) {
      send = ts + nx;
    } else {
      send = TERM | (ts + nx);               // the stream ends at nx
    }
  }
  {
    const int32_t q = (m & ~63) + lane;
    if (q >= pb && q < m) L[q] = (uint16_t)ent;
  }
  mo = m;
  return send;
}

// The candidate-exit value of a walk that ended with code `send` after m
// frame starts.
ZK_DEV int64_t ft_cx_of(int64_t send, int32_t m) {
  if (!(send & TERM)) return send | ((int64_t)m << CX_SHIFT);
  return (send & TBAD) ? FC_DEAD : FC_LIVE;
}

// Element q (wave-uniform) of a list held 64 to a register.
template <int SVN>
ZK_DEV int32_t ft_sv_at(const uint32_t (&sv)[SVN], int32_t q) {
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < SVN; ++i)
    if (i == (q >> 6)) v = sv[i];
  return __builtin_amdgcn_readlane((int)v, q & 63);
}

// The group's other tiles: the chain leaving tile t0 (end code send0; alive:
// the tile has one) walked on through them, each tile's records and its one
// candidate entry written as it goes; then the group's last exit published
// as the next group's candidate.  `nxt` holds tile t0 + 1, loaded by the
// caller (its load overlaps the caller's work).
template <int W, int G>
ZK_DEV void ft_group_tail(const FtCtx& C, int64_t send0, bool alive,
                          FtTileRegs& nxt) {
  const int lane = C.lane;
  uint8_t* sb = C.sb;
  const int64_t n = C.n, t0 = C.t;
  const int32_t maxp32 = C.maxp32;
  const int64_t ntiles = (n + FT_S - 1) / FT_S;
  // ---- the group's other tiles: the survivor's chain walked on -----------
  int64_t send = send0;
  int32_t kdone = 1;
  for (int k = 1; k < G; ++k) {
    const int64_t tk = t0 + k;
    if (tk >= ntiles) break;
    const int64_t tsk = tk * FT_S;
    const int64_t c = send;                 // the chain's entry into tk
    const bool live = alive && !(send & TERM) && c >= tsk &&
                      c < tsk + FT_S;
    if (!live) break;
    // (dbg: a walked tile's row holds its clocks — before the store, after
    // it (the load's wait), after the walk, after the records)
    int64_t* const dk = C.dbg ? C.dbg + 8 * tk : nullptr;
    const int64_t k_0 = dk ? wall_clock64() : 0;
    ft_store(sb, nxt, lane);
    const int64_t k_1 = dk ? wall_clock64() : 0;
    if (k + 1 < G && tk + 1 < ntiles) ft_load(C.buf, n, tsk + FT_S, lane, nxt);
    int32_t m;
    const int32_t nrelk = (int32_t)min(n - tsk, (int64_t)1 << 30);
    send = ft_walk(sb, (int32_t)(c - tsk), nrelk, maxp32, tsk,
                   C.list + tk * FT_LMAX, m, lane);
    const int64_t k_2 = dk ? wall_clock64() : 0;
    FcWalk wk{c, m, 0, m > 0 ? 0 : -1, false, false};
    fc_join_end(wk, send, n);
    if (lane == 0) {
      // the tile's one candidate entry: the walk's (for fs_link's chase)
      lb_store(&C.lbw[2 * (tk - 1)],
               (uint64_t)1 << 63 | (uint64_t)(c - tsk + 1));
      C.cx[5 * tk] = ft_cx_of(send, m);
      C.sx[tk] = send;
      C.rcount[tk] = m;
      C.rec_entry[tk] = c;
      C.rec_exit[tk] = wk.exit;
      C.rec_meta[tk] = fc_meta(wk);
      if (dk) {
        dk[0] = k_0;
        dk[1] = k_1;
        dk[2] = k_2;
        dk[3] = wall_clock64();
        dk[5] = (int64_t)m;
      }
    }
    if (lane >= 1 && lane < 5) C.cx[5 * tk + lane] = FC_DEAD;
    kdone = k + 1;
  }
  // tiles the walk did not reach: no entry (fs_link re-walks them)
  for (int k = kdone; k < G; ++k) {
    const int64_t tk = t0 + k;
    if (tk >= ntiles) break;
    if (lane == 0) {
      lb_store(&C.lbw[2 * (tk - 1)], (uint64_t)1 << 63);
      C.sx[tk] = -1;
      C.rcount[tk] = 0;
      C.rec_entry[tk] = -1;
      C.rec_exit[tk] = -1;
      C.rec_meta[tk] = 0;
    }
    if (lane < 5) C.cx[5 * tk + lane] = FC_DEAD;
  }
  // the group's last exit: the next group's candidate
  const int64_t tl = min(t0 + G, ntiles) - 1;
  {
    uint64_t word = (uint64_t)1 << 63;
    const int64_t tle = (tl + 1) * FT_S;
    if (kdone == (int32_t)(tl - t0 + 1) && alive && !(send & TERM) &&
        send >= tle && send < tle + W)
      word |= (uint64_t)(send - tle + 1);
    if (lane == 0) lb_store(&C.lbw[2 * tl], word);
  }
}

template <int W, int NK, int G>
ZK_DEV void fs_group_rest(const FtCtx& cx_) {
  static_assert(G > 1 && W <= 512, "groups: small windows");
  constexpr int WJ = W / 64;                // window positions per lane
  const FtCtx& C = cx_;
  const int lane = C.lane;
  uint8_t* sb = C.sb;
  const int64_t n = C.n, t0 = C.t, ts = C.ts;
  const int32_t nrel = C.nrel, maxp32 = C.maxp32, minb = C.minb;
  const int64_t ntiles = (n + FT_S - 1) / FT_S;
  FtNodes<NK> me;
  const int rounds = ft_build<NK>(me, sb, C.blk, C.pk, C.pos, C.N, nrel,
                                  maxp32, minb, lane);
  for (int k = lane; k < FT_R_B / 4; k += 64) C.sbits[k] = 0u;
  __builtin_amdgcn_wave_barrier();
  const int64_t t_f = C.dbg ? wall_clock64() : 0;

  // ---- the first tile: its preferred chain (the survivor) and its window
  // positions' roots, in registers for the entry check after the walk
  int32_t x = -1;
  const int32_t sp = ft_cands<W, false, NK>(me, sb, C.xbits, x);
  uint32_t rw[WJ];
  int64_t rx[WJ];
#pragma unroll
  for (int j = 0; j < WJ; ++j) {
    const int32_t e = lane + 64 * j;
    rw[j] = e < nrel ? ft_root_at(sb, C.blk, C.pk, e, nrel, maxp32, minb)
                     : rk(RK_END, 0, 0);
    rx[j] = e < nrel ? ft_cx(sb, rw[j], ts) : FC_LIVE;
  }
  int32_t m0 = 0;
  int64_t send0 = -1;
  uint32_t ws = 0;
  uint16_t* L0 = C.list + t0 * FT_LMAX;
  if (sp >= 0) {
    ws = ft_root_at(sb, C.blk, C.pk, sp, nrel, maxp32, minb);
    const int32_t D = ft_chain<NK>(me, sb, C.blk, C.slot, sp, ws, lane);
    if (D >= 0) {
      for (int32_t k = lane; k < D; k += 64) L0[k] = C.slot[k];
      m0 = D;
      send0 = ft_send(sb, ws, ts);
    } else {
      // (a side branch or a short frame on it: walked)
      __builtin_amdgcn_wave_barrier();
      send0 = ft_walk(sb, sp, nrel, maxp32, ts, L0, m0, lane);
      for (int32_t k = lane; k < m0; k += 64) C.slot[k] = L0[k];
      ws = 0;                  // (the slots hold the walk's starts)
    }
  }
  // the survivor's starts stay in registers (R becomes the survivor bits
  // if tile t0 has to come back)
  constexpr int SVN = (FT_SLOTS + 63) / 64;
  __builtin_amdgcn_wave_barrier();
  uint32_t sv[SVN];
#pragma unroll
  for (int i = 0; i < SVN; ++i)
    sv[i] = lane + 64 * i < m0 ? C.slot[lane + 64 * i] : 0u;
  const int64_t t_1 = C.dbg ? wall_clock64() : 0;

  FtTileRegs nxt;
  if (G > 1 && t0 + 1 < ntiles) ft_load(C.buf, n, ts + FT_S, lane, nxt);
  ft_group_tail<W, G>(C, send0, sp >= 0, nxt);

  // ---- the first tile's entry: the group before's exit -------------------
  int64_t E = 0;
  bool none = false;
  uint32_t wE = 0;
  bool known = false;          // wE / the candidate values from the table
  bool staged = false;         // tile t0 back in LDS (the fallbacks)
  auto restage = [&]() {
    if (staged) return;
    FtTileRegs r;
    ft_load(C.buf, n, ts, lane, r);
    ft_store(sb, r, lane);
    // survivor bits from the survivor's starts
    for (int k = lane; k < FT_SLOT_B / 4; k += 64) C.sbits[k] = 0u;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < SVN; ++i)
      if (lane + 64 * i < m0)
        __hip_atomic_fetch_or(&C.sbits[sv[i] >> 5], 1u << (sv[i] & 31),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __builtin_amdgcn_wave_barrier();
    staged = true;
  };
  if (t0 > 0) {
    uint64_t xw;
    int nap = 0;
    const uint64_t t_w = wall_clock64();
    for (;;) {
      xw = lb_load(&C.lbw[2 * (t0 - 1)]);
      if (xw != 0) break;
      if (wall_clock64() - t_w > FT_WAIT_TICKS) break;   // no speculation
      if (nap < 16) __builtin_amdgcn_s_sleep(2);
      else if (nap < 32) __builtin_amdgcn_s_sleep(8);
      else __builtin_amdgcn_s_sleep(32);
      ++nap;
    }
    // lane s: candidate s, looked up in the window table (the lane owning
    // position e holds its root in register e / 64)
    const int32_t v = lane < 5 ? (int32_t)((xw >> (12 * lane)) & 0xFFF) : 0;
    const bool has = v != 0 && ts + (v - 1) < n;
    const int32_t e = v - 1;
    uint32_t we = 0;
    int64_t xe = FC_DEAD;
    bool open = false;
    for (int s = 0; s < 5; ++s) {
      const int32_t es = __builtin_amdgcn_readlane(e, s);
      if (!__builtin_amdgcn_readlane((int)has, s)) continue;
      if (es >= W) {
        if (lane == s) open = true;
        continue;
      }
      const int jj = es >> 6, ll = es & 63;
      uint32_t wv = 0;
      int64_t xv = 0;
#pragma unroll
      for (int j = 0; j < WJ; ++j)
        if (j == jj) { wv = rw[j]; xv = rx[j]; }
      const uint32_t wsv = (uint32_t)__builtin_amdgcn_readlane((int)wv, ll);
      const int64_t xsv = (int64_t)(
          (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)xv,
                                                         ll) |
          (uint64_t)(uint32_t)__builtin_amdgcn_readlane(
              (int)(uint32_t)((uint64_t)xv >> 32), ll) << 32);
      if (lane == s) {
        we = wsv;
        xe = xsv;
        open = rk_kind(wsv) == RK_SHORT;
      }
    }
    if (__ballot(open)) {
      restage();
      for (uint64_t um = __ballot(open); um; um &= um - 1) {
        const int l = (int)__builtin_ctzll(um);
        const int32_t el = __builtin_amdgcn_readlane(e, l);
        const int64_t r = ft_cand(sb, C.sbits, el, nrel, maxp32, send0, n,
                                  ts, m0, lane);
        if (lane == l) xe = r;
      }
    }
    if (lane < 5) C.cx[5 * t0 + lane] = xe;
    const uint64_t hm = __ballot(has);
    const uint64_t lm = __ballot(has && xe != FC_DEAD);
    E = -1;
    if (lm) {
      const int l = (int)__builtin_ctzll(lm);
      E = ts + __builtin_amdgcn_readlane(e, l);
      wE = (uint32_t)__builtin_amdgcn_readlane((int)we, l);
      known = !__builtin_amdgcn_readlane((int)open, l);
    } else if (hm) {
      E = ts + __builtin_amdgcn_readlane(e, (int)__builtin_ctzll(hm));
    }
    none = E < 0;
  } else {
    wE = rw[0];                 // lane 0's position 0
    wE = (uint32_t)__builtin_amdgcn_readlane((int)wE, 0);
    known = true;
  }
  const int64_t t_2 = C.dbg ? wall_clock64() : 0;

  // ---- the first tile's records -------------------------------------------
  FcWalk wk{E, 0, 0, -1, false, false};
  const int32_t erel = (int32_t)(E - ts);
  bool done = false;
  if (!none && erel >= nrel) {
    fc_join_end(wk, TERM | E, n);
    done = true;
  } else if (!none && known && ws != 0 && (wE >> 16) == (ws >> 16) &&
             (int32_t)rk_cnt(wE) <= m0 && rk_cnt(wE) > 0 &&
             ft_sv_at<SVN>(sv, m0 - (int32_t)rk_cnt(wE)) == erel) {
    // the entry is on the survivor's chain: the rest is its list
    wk.js = m0 - (int32_t)rk_cnt(wE);
    wk.cnt = (int32_t)rk_cnt(wE);
    fc_join_end(wk, send0, n);
    done = true;
  }
  if (!done && !none) {
    // join: walk from the entry (tile t0 back in LDS) until the survivor's
    // path, as a single tile does
    restage();
    int64_t c = E;
    uint16_t* P = C.pre + t0 * FT_LMAX;
    int32_t np = 0;
    uint32_t ent = 0;
    const int64_t tend = ts + FT_S;
    for (;;) {
      if (c >= tend) { wk.exit = c; break; }
      if (c >= n) { wk.exit = n; break; }
      const int32_t crel = (int32_t)(c - ts);
      const uint32_t smw = C.sbits[crel >> 5];
      const int32_t lraw = lds_be32(sb, crel);
      if ((smw >> (crel & 31)) & 1u) {
        const int32_t cw = crel >> 5;
        int32_t s = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int32_t wi = lane + 64 * h;
          const uint32_t wd = C.sbits[wi];
          s += wi < cw ? __popc(wd)
                       : (wi == cw ? __popc(wd & ((1u << (crel & 31)) - 1u))
                                   : 0);
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
        wk.js = s;
        break;
      }
      const int32_t len = __builtin_amdgcn_readfirstlane(lraw);
      const int32_t nx = crel + 4 + len;
      if ((uint32_t)len > (uint32_t)maxp32 || nx > nrel) {
        wk.exit = c;
        wk.term = true;
        wk.bad = (crel + 4 <= nrel) && ((len < 0) | (len > maxp32));
        break;
      }
      ft_record(P, np, ent, crel, lane);
      c = ts + nx;
    }
    if (lane < (np & 63)) P[(np & ~63) + lane] = (uint16_t)ent;
    wk.np = np;
    wk.cnt = np;
    if (wk.js >= 0) {
      wk.cnt = np + (m0 - wk.js);
      fc_join_end(wk, send0, n);
    }
  } else if (none) {
    if (m0 > 0) fc_join_end(wk, send0, n);
    if (lane == 0) fc_stat(C.stats, 1, 1), fc_stat(C.stats, LW_NOSPEC, 1);
  }
  if (lane == 0) {
    C.sx[t0] = send0;
    C.rcount[t0] = m0;
    C.rec_entry[t0] = none ? -1 : E;
    C.rec_exit[t0] = wk.exit;
    C.rec_meta[t0] = fc_meta(wk);
    if (C.dbg) {
      int64_t* d = C.dbg + 8 * t0;
      d[0] = C.t_0;
      d[1] = t_1;
      d[2] = t_2;
      d[3] = wall_clock64();
      d[4] = C.t_d;
      d[5] = (int64_t)C.N | (int64_t)rounds << 16 | (int64_t)done << 24;
      d[6] = C.t_s;
      d[7] = t_f;
    }
  }
}

template <int W, bool LONG, int G>
__global__ __launch_bounds__(256) void fs_tile(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ n_dev,
    int64_t n_cap, int64_t maxp, uint16_t* __restrict__ list,
    uint16_t* __restrict__ pre, int64_t* __restrict__ sx, uint64_t* lbw,
    int64_t* __restrict__ rec_entry, int64_t* __restrict__ rec_exit,
    int64_t* __restrict__ rec_meta, int32_t* __restrict__ rcount,
    int64_t ntiles_cap, int64_t* __restrict__ dbg, int32_t minb,
    int32_t tflags, int64_t* __restrict__ cx) {
  static_assert(W % 64 == 0 && W <= 2048, "window");
  // one tile per wave; a block's waves work independently (no barriers),
  // each in its own LDS slice
  extern __shared__ __attribute__((aligned(16))) uint8_t smem_all[];
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint8_t* smem = smem_all + wv * FT_LDS;
  FtCtx C;
  C.sb = smem;
  uint64_t* bmask = (uint64_t*)(smem + FT_O_BLK);
  uint16_t* bbase = (uint16_t*)(smem + FT_O_BASE);
  C.blk.mask = bmask;
  C.blk.base = bbase;
  C.pk = (uint32_t*)(smem + FT_O_PK);
  C.pos = (uint16_t*)(smem + FT_O_R);
  C.slot = (uint16_t*)(smem + FT_O_R);
  C.sbits = (uint32_t*)(smem + FT_O_R);
  C.xbits = (uint32_t*)(smem + FT_O_XB);
  const int lane = threadIdx.x & 63;
  const int64_t n = stream_len(n_dev, n_cap);
  const int64_t ntiles = (n + FT_S - 1) / FT_S;
  // (tiles in workgroup order: a tile's predecessor was dispatched before
  // it.  An XCD-by-XCD mapping — each XCD a contiguous tile range — put
  // the predecessor on the same L2 but started every range's tail later:
  // reply stream 94 -> 103 us.)
  const int64_t t = ((int64_t)blockIdx.x * (blockDim.x >> 6) + wv) * G;
  if (t >= ntiles) return;
  C.t_0 = dbg ? wall_clock64() : 0;
  const int64_t ts = t * FT_S;
  const int64_t tend = ts + FT_S;
  const int32_t nrel = (int32_t)min(n - ts, (int64_t)1 << 30);
  const int32_t maxp32 = (int32_t)maxp;
  uint8_t* sb = C.sb;

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
#pragma unroll
    for (int j = 0; j < PER; ++j) *(uint4*)(sb + 16 * (lane + 64 * j)) = v[j];
    if (lane == 0) *(uint4*)(sb + FT_S) = pad;
  }
  __builtin_amdgcn_wave_barrier();
  C.t_s = dbg ? (__builtin_amdgcn_s_waitcnt(0), wall_clock64()) : 0;

  // ---- 1. nodes: lane l tests positions 64l .. 64l + 63 ------------------
  int32_t N;
  {
    const int32_t P0 = lane * 64;
    uint32_t d[17];
    {
      // lane l reads its 16-byte chunks in the order rotated by (l >> 2) & 3:
      // a ds_read_b128 lane group (16 lanes) then covers the 64 banks once
      // (in plain order four lanes share each 16-byte slot: 4-way); the
      // dword past the lane's 64 bytes is the next lane's first (a shuffle,
      // not a 16-way ds_read_b32 at a 64-byte stride)
      const int r = (lane >> 2) & 3;
      uint4 x0 = *(const uint4*)(sb + P0 + 16 * (r & 3));
      uint4 x1 = *(const uint4*)(sb + P0 + 16 * ((1 + r) & 3));
      uint4 x2 = *(const uint4*)(sb + P0 + 16 * ((2 + r) & 3));
      uint4 x3 = *(const uint4*)(sb + P0 + 16 * ((3 + r) & 3));
      const uint32_t pad = *(const uint32_t*)(sb + FT_S);   // (broadcast)
      // back to chunk order (x_j held chunk j + r): rotate right by r in two
      // conditional stages (named registers and selects: an indexed array
      // went to scratch)
      auto sel = [](bool c, uint4 a, uint4 b) {
        return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z,
                          c ? a.w : b.w);
      };
      {
        const bool c = r & 1;
        const uint4 y0 = sel(c, x3, x0), y1 = sel(c, x0, x1),
                    y2 = sel(c, x1, x2), y3 = sel(c, x2, x3);
        x0 = y0; x1 = y1; x2 = y2; x3 = y3;
      }
      {
        const bool c = r & 2;
        const uint4 y0 = sel(c, x2, x0), y1 = sel(c, x3, x1),
                    y2 = sel(c, x0, x2), y3 = sel(c, x1, x3);
        x0 = y0; x1 = y1; x2 = y2; x3 = y3;
      }
      d[0] = x0.x; d[1] = x0.y; d[2] = x0.z; d[3] = x0.w;
      d[4] = x1.x; d[5] = x1.y; d[6] = x1.z; d[7] = x1.w;
      d[8] = x2.x; d[9] = x2.y; d[10] = x2.z; d[11] = x2.w;
      d[12] = x3.x; d[13] = x3.y; d[14] = x3.z; d[15] = x3.w;
      const uint32_t nx = (uint32_t)__shfl_down((int)d[0], 1, 64);
      d[16] = lane == 63 ? pad : nx;
    }
    // minb <= len <= W - 4 past the entry window (the window covers the
    // stream's frames: a longer length is a byte pattern, not a frame; the
    // rare real one meets the map as a SHORT root and is walked exactly),
    // len < FT_LIMIT in long-frame mode; in the entry window any legal
    // length (a frame there longer than the tile is still an entry's
    // chain).  (Length-like words inside frames — zxids in [2^27, 2^28)
    // read 2048..4095 — took a create / set / delete reply tile past
    // FT_NMAX nodes: no map, no speculation, a 200 ms serial repair.)
    const uint32_t lim = P0 < W ? (uint32_t)(maxp32 - minb + 1)
                         : LONG ? (uint32_t)(FT_LIMIT - minb)
                                : (uint32_t)(W - 3 - minb);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const uint32_t v = (uint32_t)be32_of(d[j >> 2], d[(j >> 2) + 1], j);
      lo |= ((v - (uint32_t)minb) < lim ? 1u : 0u) << j;
    }
#pragma unroll
    for (int j = 32; j < 64; ++j) {
      const uint32_t v = (uint32_t)be32_of(d[j >> 2], d[(j >> 2) + 1], j);
      hi |= ((v - (uint32_t)minb) < lim ? 1u : 0u) << (j - 32);
    }
    uint64_t mask = (uint64_t)hi << 32 | lo;
    // a node's length word lies inside the stream
    const int32_t room = nrel - 4 - P0;      // last position with a header
    if (room < 63) mask = room < 0 ? 0 : mask & ((2ull << room) - 1);
    const uint32_t c = (uint32_t)__popcll(mask);
    uint32_t incl = c;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      const uint32_t y = __shfl_up(incl, s, 64);
      if (lane >= s) incl += y;
    }
    N = __builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t base = incl - c;
    bmask[lane] = mask;
    bbase[lane] = (uint16_t)base;
    if (N <= FT_NMAX) {
      uint32_t k = base;
      uint64_t m = mask;
      while (m) {
        C.pos[k++] = (uint16_t)(P0 + __builtin_ctzll(m));
        m &= m - 1;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  C.t_d = dbg ? wall_clock64() : 0;
  C.buf = buf; C.list = list; C.pre = pre; C.sx = sx; C.lbw = lbw;
  C.rec_entry = rec_entry; C.rec_exit = rec_exit; C.rec_meta = rec_meta;
  C.rcount = rcount; C.dbg = dbg; C.cx = cx;
  C.stats = &lbw[2 * ntiles_cap];
  C.n = n; C.t = t; C.ts = ts; C.tend = tend;
  C.nrel = nrel; C.maxp32 = maxp32; C.minb = minb; C.N = N;
  C.nospec = tflags & 1;
  C.misspec = tflags >> 8;
  C.lane = lane;
  // ---- 2-5, with this lane's share of the nodes in registers -------------
  static_assert(FT_NMAX == 512, "node buckets");
  if constexpr (G > 1) {
    static_assert(!LONG, "groups: frames within the window");
    if (N <= 128) fs_group_rest<W, 2, G>(C);
    else if (N <= 256) fs_group_rest<W, 4, G>(C);
    else if (N <= FT_NMAX) fs_group_rest<W, 8, G>(C);
    else {
      // no map for the first tile (its candidates walked lane by lane):
      // its survivor's exit is walked on through the group as usual
      const int64_t s0 = fs_tile_rest<W, LONG, 1>(C, false);
      FtTileRegs nxt;
      if (t + 1 < (n + FT_S - 1) / FT_S) ft_load(buf, n, ts + FT_S, lane, nxt);
      ft_group_tail<W, G>(C, s0, s0 >= 0, nxt);
    }
  } else {
    if (N <= 128) fs_tile_rest<W, LONG, 2>(C, true);
    else if (N <= 256) fs_tile_rest<W, LONG, 4>(C, true);
    else if (N <= FT_NMAX) fs_tile_rest<W, LONG, 8>(C, true);
    else fs_tile_rest<W, LONG, 1>(C, false);
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
// through a WIN-byte LDS window (4 KiB per wave: a tile in one staging).
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

// fs_link's grid: fl_blocks() workgroups check the links (fl_check), then
// each takes a ticket; the LAST block to arrive reads the check's minima
// and does the rest alone.  No block ever waits for another, so nothing
// depends on the grid being co-resident: a spin barrier here (rounds 2-4)
// waited for room beside the other connection's kernels (34 us in the
// overlapped GET step against 12 us alone, one 175 ms step on the watch
// stream).  The usual scan — no broken link before the first terminal —
// is the bases scan.  A repair: a handful of broken links are chased in
// parallel waves (fl_chase); more (every tile without a speculated entry,
// a run of garbage entries) go to the tail, which chases from the leftmost
// broken link with the exact entry — one wave looks a run of tiles up in
// fs_tile's candidate exits 64 at a time, walking only the tiles whose
// exact entry is not a candidate — until every live link holds.
// Before its ticket, a block re-walks the broken links its own check found
// (one wave a link, from the exit before it as recorded; fl_accept's rule),
// one parallel repair round over the whole grid without any barrier: a
// tile whose speculated entry was missing or wrong but whose survivor is
// the true chain (every tile of a `nospec` stream, a frontier wait that
// timed out) re-walks to the same exit, so the round settles any number of
// such tiles at once — the last block then only checks and re-counts.
// Grid words (LW_GRID, uint64): [0] the ticket, [1] tiles the blocks
// re-walked, [FL_NB] the check's count of broken links (fs_rows clears it
// for the next scan).
// At most this many broken links: chased from the check's list (fl_chase; a
// reply stream usually has a handful of broken links or none); more go to
// the tail's exact chases.
constexpr unsigned long long FL_SMALL = 1024;

ZK_DEV int64_t rfl64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Is a repair walk of tile k (new exit x) written?  Always when the link
// before k holds (its entry E is then exact, or at least as good as the
// records get).  When that link is itself broken, E is suspect: a garbage
// exit of tile k-1 (say a frame-length read from an xid, megabytes ahead)
// walked on would break the link after k where it holds, that link's walk
// would break the next, and a wave of garbage would cross the stream one
// tile per round (the first storm reply stream: 1413 tiles re-walked over
// 71 rounds).  So a suspect walk that changes the exit is not written while
// link k+1 holds; link k stays broken for the last block's chases.  A walk
// from an E that tile k-1 has since replaced (another wave re-walked it at
// the same time) is stale and not written either.  (A refused walk has
// overwritten the tile's recorded frame starts all the same: its caller
// clears the entry.)
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

// The block's repair round (see FL_LOC): its check's broken links, one wave
// a link.  Returns the tiles this wave re-walked.
ZK_DEV uint32_t fl_local_round(const uint8_t* __restrict__ buf, int64_t n,
                               int64_t ntiles, int64_t maxp,
                               const int64_t* __restrict__ sx,
                               const uint16_t* __restrict__ list,
                               const int32_t* __restrict__ rcount,
                               uint16_t* pre, int64_t* rec_entry,
                               int64_t* rec_exit, int64_t* rec_meta,
                               const int32_t* lloc, int nloc, uint8_t* win) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint8_t* mywin = win + (size_t)wv * (FC_WIN + 16);
  uint32_t walked = 0;
  for (int j = wv; j < nloc; j += FL_T / 64) {
    const int64_t k = lloc[j];
    const int64_t E = rfl64(ld_agent(&rec_exit[k - 1]));
    if (E < k * FT_S ||
        __builtin_amdgcn_readfirstlane(m_term(ld_agent(&rec_meta[k - 1]))))
      continue;                               // no usable entry yet
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
        st_agent(&rec_entry[k], -1);
      }
    }
  }
  return walked;
}

// ---- the big repair ---------------------------------------------------------
// A scan with hundreds of tiles without a speculated entry (adversarial
// streams: every payload word a plausible length, tests that withhold
// every entry) needs the grid's parallelism round after round, which no
// single block has: there the grid keeps the barrier rounds of rounds 2-4.
// The decision comes from fs_tile's count of this scan, known before
// fs_link starts, so every block takes the same path and no ordinary scan
// ever waits in a barrier.  Barrier words (LW_BIG, uint64): [0] arrivals,
// [1] generation, [2] abort, [4 + 2r] the links round r listed.
constexpr uint64_t FL_BAR_TICKS = 50000000;   // 0.5 s: barrier abandoned

// Grid barrier over fs_link's workgroups (16: they find CUs beside
// anything else that runs, and nothing they wait for needs a CU they hold).
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

// The full check (fs_link, when fs_tile counted a bad link): every link and

// The full check (fs_link, when fs_tile counted a bad link): every link and
// terminal, one wave per count block of FK_T tiles over the grid, and the
// frame counts scanned per block: base[k] = count before tile k within its
// block, bsum[b] = the block's total.  The leftmost broken link and terminal
// go to mins[0..1] as (ntiles - k) maxima, the broken links to blist (their
// count in *nbroken).  Cross-block data: agent-scope stores (the blocks may
// sit on different XCDs, each with its own L2).
ZK_DEV void fl_check(int64_t ntiles, const int64_t* __restrict__ rec_entry,
                     const int64_t* __restrict__ rec_exit,
                     const int64_t* __restrict__ rec_meta, int64_t* base,
                     int64_t* bsum, uint64_t* mins,
                     unsigned long long* nbroken, int32_t* blist,
                     int32_t* lloc, int* lcnt) {
  const int lane = threadIdx.x & 63;
  const int64_t INF = INT64_MAX;
  const int64_t nw = (int64_t)gridDim.x * (FL_T / 64);
  const int64_t nbl = (ntiles + FK_T - 1) / FK_T;
  int64_t fb = INF, fterm = INF;
  for (int64_t b = (int64_t)blockIdx.x * (FL_T / 64) + (threadIdx.x >> 6);
       b < nbl; b += nw) {
    const int64_t k = b * FK_T + lane;
    int64_t cnt = 0;
    bool brk = false;
    if (k < ntiles) {
      // written by fs_tile (an earlier launch): plain loads, issued together
      const int64_t mk = rec_meta[k];
      const bool nxt = k + 1 < ntiles;
      const int64_t e = nxt ? rec_entry[k + 1] : 0;
      const int64_t x = rec_exit[k];
      cnt = m_cnt(mk);
      if (m_term(mk)) {
        fterm = min(fterm, k);
      } else if (nxt && (e < 0 || e != x)) {
        brk = true;
        fb = min(fb, k + 1);
      }
    }
    const uint64_t bm = __ballot(brk);
    if (bm) {
      unsigned long long b0 = 0;
      if (lane == 0) b0 = atomicAdd(nbroken, (unsigned long long)__popcll(bm));
      b0 = __shfl(b0, 0, 64);
      int l0 = 0;
      if (lane == 0) l0 = atomicAdd(lcnt, __popcll(bm));
      l0 = __shfl(l0, 0, 64);
      if (brk) {
        const uint64_t below = lane ? (bm & ((~0ull) >> (64 - lane))) : 0ull;
        __hip_atomic_store(&blist[b0 + __popcll(below)], (int32_t)(k + 1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int li = l0 + __popcll(below);
        if (li < FL_LOC) lloc[li] = (int32_t)(k + 1);
      }
    }
    int64_t inc = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t v = __shfl_up(inc, d, 64);
      if (lane >= d) inc += v;
    }
    if (k < ntiles) st_agent(&base[k], inc - cnt);
    if (lane == 63) st_agent(&bsum[b], inc);
  }
  for (int d = 32; d >= 1; d >>= 1) {
    fb = min(fb, (int64_t)__shfl_xor(fb, d, 64));
    fterm = min(fterm, (int64_t)__shfl_xor(fterm, d, 64));
  }
  if (lane == 0) {
    if (fb != INF) atomicMax((unsigned long long*)&mins[0],
                             (unsigned long long)(ntiles - fb));
    if (fterm != INF) atomicMax((unsigned long long*)&mins[1],
                                (unsigned long long)(ntiles - fterm));
  }
}

// Row bases once every link up to the first terminal ft (INF: none) holds:
// bsum[b] (block b's count total, the check's or re-counted) becomes block
// b's exclusive offset; base[k] stays the in-block one; result[0..3] and
// the last tile.  fs_link's last block alone.
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
// The check listed the broken links.  A chase starts at one with the exact
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
// fs_link's tail (exact chases from the leftmost broken link) finishes from
// the records as they stand.
constexpr int FL_WL = 1024;                // chases per round
constexpr int FL_HS = 2048;                // their dedup hash set
constexpr int FL_WR = 48;                  // rounds before the tail
constexpr int FL_DB = 8192;                // count blocks tracked (2M tiles)
static_assert(FL_SMALL <= FL_WL, "the check's list fits the first round");

struct FlChase {
  uint32_t* dirty;                // count blocks holding re-written tiles
  int* overflow;
  uint64_t* stats;
  int64_t* clk;                   // ZKMI_FS_DBG: the exact chase's span
};

ZK_DEV void fl_dirty(FlChase& ch, int64_t t) {
  const int64_t b = t / FK_T;
  // (past FL_DB count blocks only the tail chases, which re-counts all)
  if (b < FL_DB) atomicOr(&ch.dirty[b >> 5], 1u << (b & 31));
}

ZK_DEV int live_count(const int64_t* c5) {
  int live = 0;
#pragma unroll
  for (int j = 0; j < 5; ++j) live += c5[j] != FC_DEAD;
  return live;
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
// chase writes nothing that would break a link that holds (a phantom's
// exit must not run over a true segment: a garbage exit walked on would
// break the link after it, and a wave of garbage would cross the stream one
// tile per round); it stops there and the link waits for a later round.
ZK_DEV int64_t fl_chase_run(const uint8_t* __restrict__ buf, int64_t n,
                            int64_t ntiles, int64_t maxp,
                            const int64_t* __restrict__ sx,
                            const uint16_t* __restrict__ list,
                            const int32_t* __restrict__ rcount, uint16_t* pre,
                            int64_t* rec_entry, int64_t* rec_exit,
                            int64_t* rec_meta, const uint64_t* lbw,
                            const int64_t* cx,
                            uint8_t* mywin, FlChase& ch, int64_t k0,
                            bool exact, bool& term, uint32_t& walked,
                            uint32_t walk_budget = 0) {
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
      // (a budgeted chase leaves the walking to the caller's rounds)
      if (walk_budget != 0 && walked >= walk_budget) return t - 1;
      const int32_t m0 = __builtin_amdgcn_readfirstlane(rcount[t]);
      const FcWalk fw = fc_walk(buf, n, maxp, ts, E, list + t * FT_LMAX, m0,
                                sx[t], mywin, pre + t * FT_LMAX, lane);
      ++walked;
      if (!exact && rfl64(fw.exit) != oldx && nh) {
        // refused, but the walk overwrote the tile's frame starts (pre)
        // while its record keeps the old entry: no entry, so its link stays
        // broken and the tile is walked again
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

// fs_link's last block: chase rounds to a fix-point of the links.  Returns false when it
// gave up (the tail takes over).
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
  // the check's list to LDS
  for (int i = tid; i < nb0; i += FL_T)
    wl[0][i] = __hip_atomic_load(&blist[i], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
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

// After the chases and the check of every link (the last block): re-count
// the count blocks holding a re-written tile, one wave per block, a tile per
// lane.
ZK_DEV void fl_chase_recount(int64_t ntiles, const int64_t* rec_meta,
                             int64_t* base, int64_t* bsum, FlChase& ch) {
  static_assert(FK_T == 64, "a count block is a wave");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nbl = (ntiles + FK_T - 1) / FK_T;
  for (int64_t b = wv; b < nbl; b += FL_T / 64) {
    if (!((ch.dirty[b >> 5] >> (b & 31)) & 1u)) continue;
    const int64_t k = b * FK_T + lane;
    const int64_t c = k < ntiles ? m_cnt(ld_agent(&rec_meta[k])) : 0;
    int64_t inc = c;
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t v = __shfl_up(inc, d, 64);
      if (lane >= d) inc += v;
    }
    if (k < ntiles) st_agent(&base[k], inc - c);
    if (lane == 63) st_agent(&bsum[b], inc);
  }
  __syncthreads();
}

// Every live link holds up to the first terminal ft (INF: none): the
// exclusive scan of the counts of tiles 0..ft as absolute row bases (bsum
// zero: fs_rows adds no block offset), tiles after ft dead; result[0..3]
// and the last tile.  The last block alone, after a repair.
ZK_DEV void fl_count_scan(int64_t n, int64_t ntiles, int64_t ft,
                          const int64_t* rec_exit, const int64_t* rec_meta,
                          int64_t* base, int64_t* bsum, int64_t cap,
                          int64_t* result, int64_t* lastk, int64_t* red) {
  const int tid = threadIdx.x;
  const int64_t INF = INT64_MAX;
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
  for (int64_t b = tid; b <= last / FK_T; b += FL_T) bsum[b] = 0;
  if (tid == 0) {
    *lastk = last;
    result[0] = tot;
    result[3] = tot > cap ? 1 : 0;
    if (ft == INF) {
      result[1] = n;
      result[2] = 0;
    } else {
      // (a stop before a tile that is no terminal — unreachable, see the
      // tail — leaves the carry at tile ft's exit)
      const int64_t mf = ld_agent(&rec_meta[ft]);
      result[1] = ld_agent(&rec_exit[ft]);
      result[2] = m_term(mf) && m_bad(mf) ? 1 : 0;
    }
  }
}

// The leftmost terminal, and the leftmost broken link at or after `from`
// (INF: none), over the whole block.  Loads in batches of FL_U tiles a
// thread, all issued before any is used (one round trip a batch).
ZK_DEV void fl_links(int64_t from, int64_t ntiles,
                     const int64_t* rec_entry, const int64_t* rec_exit,
                     const int64_t* rec_meta, int64_t* red, int64_t& fb_out,
                     int64_t& ft_out) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t INF = INT64_MAX;
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
  fb_out = fb;
  ft_out = fterm;
}

// Every broken link (after a tile that is no terminal) into blist, in tile
// order, by the whole block; returns their count.  fb / ft: the leftmost
// broken link and terminal (INF: none).
ZK_DEV int64_t fl_list_broken(int64_t ntiles, const int64_t* rec_entry,
                              const int64_t* rec_exit, const int64_t* rec_meta,
                              int32_t* blist, int64_t* red, int64_t& fb_out,
                              int64_t& ft_out) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t INF = INT64_MAX;
  // a thread's run of tiles, its loads in batches of FL_U (all issued
  // before any is used) — this runs once per repair round
  const int64_t per = (ntiles + FL_T - 1) / FL_T;
  const int64_t k0 = (int64_t)tid * per, k1 = min(k0 + per, ntiles);
  int64_t cnt = 0, fb = INF, fterm = INF;
  for (int pass = 0; pass < 2; ++pass) {
    int64_t w = 0;
    if (pass == 1) {
      int64_t tot;
      w = block_excl_scan(cnt, red, &tot);
      red[2 * (FL_T / 64) + 1] = tot;       // (read after the loop)
      if (cnt == 0) break;
    }
    for (int64_t kb = k0; kb < k1; kb += FL_U) {
      int64_t mp[FL_U], mk[FL_U], e[FL_U], x[FL_U];
#pragma unroll
      for (int u = 0; u < FL_U; ++u) {
        const int64_t k = kb + u;
        const bool in = k < k1;
        mk[u] = in ? ld_agent(&rec_meta[k]) : 0;
        mp[u] = in && k >= 1 ? ld_agent(&rec_meta[k - 1]) : 0;
        e[u] = in ? ld_agent(&rec_entry[k]) : 0;
        x[u] = in && k >= 1 ? ld_agent(&rec_exit[k - 1]) : 0;
      }
#pragma unroll
      for (int u = 0; u < FL_U; ++u) {
        const int64_t k = kb + u;
        if (k >= k1) break;
        const bool brk = k >= 1 && !m_term(mp[u]) && e[u] != x[u];
        if (pass == 0) {
          if (brk) { ++cnt; fb = min(fb, k); }
          if (m_term(mk[u])) fterm = min(fterm, k);
        } else if (brk) {
          blist[w++] = (int32_t)k;
        }
      }
    }
  }
  __syncthreads();
  const int64_t total = red[2 * (FL_T / 64) + 1];
  __syncthreads();
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
  fb_out = fb;
  ft_out = fterm;
  return total;
}

__global__ __launch_bounds__(FL_T) void fs_link(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ n_dev,
    int64_t n_cap, int64_t maxp, const int64_t* __restrict__ sx,
    const uint16_t* __restrict__ list, const int32_t* __restrict__ rcount,
    uint16_t* pre, int64_t* rec_entry, int64_t* rec_exit, int64_t* rec_meta,
    int64_t* __restrict__ base, int64_t cap, int64_t* __restrict__ result,
    uint64_t* stats, int32_t* __restrict__ blist,
    int64_t* __restrict__ bsum, uint64_t* mins,
    int64_t* __restrict__ lastk, unsigned long long* g,
    const uint64_t* lbw, const int64_t* __restrict__ cx,
    int64_t* __restrict__ ldbg, int32_t local_min, int32_t fflags) {
  __shared__ __attribute__((aligned(16)))
      uint8_t win[(FL_T / 64) * (FC_WIN + 16)];      // one per wave
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
  const int64_t t_in = ldbg != nullptr ? wall_clock64() : 0;
  // the check over the grid (links, terminals, in-block counts; a launch of
  // its own until round 4), the block's repair round over the broken links
  // it found, then a ticket: the last block to take one sees every block's
  // check and repairs (each releases them before its ticket) and goes on
  // alone; the others are done
  __shared__ int32_t lloc[FL_LOC];
  __shared__ int s_lcnt;
  if (tid == 0) s_lcnt = 0;
  __syncthreads();
  fl_check(ntiles, rec_entry, rec_exit, rec_meta, base, bsum, mins, &g[FL_NB],
           blist, lloc, &s_lcnt);
  if (ldbg != nullptr && tid == 0 && blockIdx.x < FL_DBG_BLOCKS) {
    // (ZKMI_FS_DBG: every block's entry and check-done clocks, rows 1-4 of
    // fs_link's debug rows)
    ldbg[8 + 2 * blockIdx.x] = t_in;
    ldbg[8 + 2 * blockIdx.x + 1] = wall_clock64();
  }
  // the big repair (see FL_BIG_NOSPEC): barrier rounds over the grid, then
  // block 0 goes on as the last block does
  const bool big = (uint32_t)ld_agent((const int64_t*)&stats[LW_NOSPEC]) >
                   FL_BIG_NOSPEC;
  if (big) {
    unsigned long long* gb = (unsigned long long*)(stats + LW_BIG);
    bool ok = fl_sync(gb);
    for (int r = 0; r < FL_GROUNDS && ok; ++r)
      ok = fl_round(buf, n, ntiles, maxp, sx, list, rcount, pre, rec_entry,
                    rec_exit, rec_meta, blist, gb, r, red, win, stats);
    if (blockIdx.x != 0) return;
    __syncthreads();
    if (tid == 0) {
      gb[2] = 0;
      for (int r = 0; r < FL_GROUNDS; ++r) gb[4 + 2 * r] = 0;
    }
  }
  __syncthreads();
  // (a handful of broken links — a frontier timeout, a garbage candidate,
  // the ends of a phantom chain's region — are the last block's chases:
  // an exact chase runs on through a region of consistent-but-wrong links
  // that no per-link walk sees broken)
  if (!big && s_lcnt > local_min) {
    const uint32_t w = fl_local_round(buf, n, ntiles, maxp, sx, list, rcount,
                                      pre, rec_entry, rec_exit, rec_meta, lloc,
                                      min(s_lcnt, FL_LOC), win);
    if (lane == 0 && w) {
      fc_stat(stats, 2, w);
      atomicAdd(&g[1], (unsigned long long)w);
    }
  }
  __shared__ int s_last;
  __syncthreads();
  if (big) {
    if (tid == 0) s_last = 1;             // (block 0, after the rounds)
  } else if (tid == 0) {
    __threadfence();
    const unsigned long long a = __hip_atomic_fetch_add(
        &g[0], 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    const int last = a + 1 == gridDim.x;
    // the ticket back to zero for the next scan of this workspace
    if (last)
      __hip_atomic_store(&g[0], 0ull, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  // the minima and the broken-link count (fs_rows clears them for the next
  // scan of this workspace), and the tiles the blocks' rounds re-walked
  const uint64_t mb0 = ld_agent((const int64_t*)&mins[0]);
  const uint64_t mt0 = ld_agent((const int64_t*)&mins[1]);
  const unsigned long long nb0 = __hip_atomic_load(
      &g[FL_NB], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long rew = __hip_atomic_load(
      &g[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int64_t fb0 = mb0 ? ntiles - (int64_t)mb0 : INF;
  const int64_t ft0 = mt0 ? ntiles - (int64_t)mt0 : INF;
  if (!big && (fb0 == INF || fb0 > ft0)) {
    // no broken link before the first terminal (the blocks re-walked only
    // links past it, whose counts no row uses): the row bases are bsum's
    // block offsets + the check's in-block bases
    if (ldbg != nullptr && tid == 0) ldbg[40] = wall_clock64();
    fl_bases(n, ntiles, ft0, rec_exit, rec_meta, base, bsum, cap, result,
             lastk, red);
    if (tid == 0 && rew) g[1] = 0;
    if (ldbg != nullptr && tid == 0) ldbg[41] = wall_clock64();
    return;
  }
  if (tid == 0) g[1] = 0;
  __shared__ uint32_t dirty[FL_DB / 32];
  __shared__ int s_ovf;
  FlChase ch{dirty, &s_ovf, stats, ldbg};
  for (int i = tid; i < FL_DB / 32; i += FL_T) dirty[i] = 0;
  if (tid == 0) s_ovf = 0;
  __syncthreads();
  const bool clk = ldbg != nullptr && tid == 0;
  // (ZKMI_FS_DBG: [5] the last block's start, [4] the end | path << 56:
  // 1 chases, 2 count scan after rounds, 3 tail)
  if (clk) ldbg[5] = t_in;
  int64_t from = 1, ft = INF;
  int64_t nb = (int64_t)nb0;
  // repair rounds of this block: a handful of broken links are chased (the
  // usual repair: one pass, then only the count blocks it touched are
  // re-counted); many are re-walked in parallel, one wave a link (the
  // blocks' round continued here); after each, the links still broken are
  // listed again.  What the rounds leave goes to the tail.
  bool changed = rew != 0 || big;       // records changed beyond the chases' dirty
  if (!big && nb > (int64_t)FL_SMALL && fb0 != INF && (fflags & 1)) {
    // many broken links: first ONE exact chase from the leftmost, wave 0,
    // through fs_tile's candidate exits 64 tiles a batch.  A stream whose
    // every frame carries a phantom chain of the frame's own period (SET_DATA
    // replies of version 84: both chains survive every tile, about half the
    // tiles speculate the phantom) is settled by it in one pass of lookups
    // (ms) where the rounds walked every broken tile (84 ms a scan).  Its
    // walks are budgeted: on a stream whose entries are not candidates
    // (dense payload words) it stops early and the rounds walk in parallel
    // (profiles/r5_fs_link_ab.md).  Not after the grid's big repair.
    if (wv == 0) {
      bool term = false;
      uint32_t walked = 0;
      const int64_t kend = fl_chase_run(buf, n, ntiles, maxp, sx, list, rcount,
                                        pre, rec_entry, rec_exit, rec_meta, lbw,
                                        cx, win, ch, fb0, true, term, walked,
                                        FL_CHASE_WALKS);
      (void)kend;
      if (lane == 0) {
        if (walked) fc_stat(stats, 2, walked);
        fc_stat(stats, 3, 1);
      }
    }
    __syncthreads();
    changed = true;
  }
  for (int round = 0; round < FL_BROUNDS; ++round) {
    if (changed) {
      int64_t fbv, ftv;
      nb = fl_list_broken(ntiles, rec_entry, rec_exit, rec_meta, blist, red,
                          fbv, ftv);
      if (fbv == INF || fbv > ftv) {
        fl_count_scan(n, ntiles, ftv, rec_exit, rec_meta, base, bsum, cap,
                      result, lastk, red);
        if (clk) ldbg[4] = wall_clock64() | (2ll << 56);
        return;
      }
    }
    if (nb <= (int64_t)FL_SMALL && (ntiles + FK_T - 1) / FK_T <= FL_DB) {
      // ---- a handful of broken links: chases, then every link checked ---
      if (clk && round == 0) ldbg[0] = wall_clock64();
      const bool settled = fl_chase(buf, n, ntiles, maxp, sx, list, rcount,
                                    pre, rec_entry, rec_exit, rec_meta, lbw,
                                    cx, blist, (int)nb, win, stats, ch);
      if (clk && round == 0) ldbg[1] = ldbg[2] = wall_clock64();
      // a chase only vouches for the links it saw
      int64_t fbv, ftv;
      fl_links(1, ntiles, rec_entry, rec_exit, rec_meta, red, fbv, ftv);
      if (clk && round == 0) ldbg[3] = wall_clock64();
      if (settled && (fbv == INF || fbv > ftv)) {
        if (changed) {
          // (tiles re-walked in rounds are not in the chases' dirty set)
          fl_count_scan(n, ntiles, ftv, rec_exit, rec_meta, base, bsum, cap,
                        result, lastk, red);
          if (clk) ldbg[4] = wall_clock64() | (2ll << 56);
          return;
        }
        fl_chase_recount(ntiles, rec_meta, base, bsum, ch);
        fl_bases(n, ntiles, ftv, rec_exit, rec_meta, base, bsum, cap, result,
                 lastk, red);
        if (clk) ldbg[4] = wall_clock64() | (1ll << 56);
        return;
      }
      if (!settled) break;              // the lists outgrew LDS: the tail
    } else {
      const uint32_t w = fl_local_round(buf, n, ntiles, maxp, sx, list,
                                        rcount, pre, rec_entry, rec_exit,
                                        rec_meta, blist, (int)nb, win);
      if (lane == 0 && w) fc_stat(stats, 2, w);
      if (tid == 0) fc_stat(stats, 3, 1);
      __syncthreads();
    }
    changed = true;
  }
  // ---- the tail: exact chases from the leftmost broken link, until every
  // live link holds; then the count scan ------------------------------------
  for (;;) {
    int64_t fb, fterm;
    fl_links(from, ntiles, rec_entry, rec_exit, rec_meta, red, fb, fterm);
    // terminals before from - 1 were found in an earlier pass of this loop
    // (links before `from` hold)
    if (fb == INF || fb > fterm) {          // every live link holds
      ft = fterm;
      break;
    }
    if (wv == 0) {
      // the leftmost broken link has the exact entry (the exit before it):
      // the chase settles tile fb at least (looked up or walked)
      bool term = false;
      uint32_t walked = 0;
      const int64_t kend = fl_chase_run(buf, n, ntiles, maxp, sx, list, rcount,
                                        pre, rec_entry, rec_exit, rec_meta, lbw,
                                        cx, win, ch, fb, true, term, walked);
      if (lane == 0) {
        // (kend < fb: nothing written, which the records before fb rule out;
        // the scan then stops before tile fb rather than loop)
        s_next = kend < fb ? -fb : kend + 1;
        if (walked) fc_stat(stats, 2, walked);
        fc_stat(stats, 3, 1);
      }
    }
    __syncthreads();
    from = s_next;
    __syncthreads();
    if (from < 0) {
      ft = -from - 1;
      break;
    }
  }
  fl_count_scan(n, ntiles, ft, rec_exit, rec_meta, base, bsum, cap, result,
                lastk, red);
  if (clk) ldbg[4] = wall_clock64() | (3ll << 56);
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
    int32_t* __restrict__ flen, int64_t cap, uint64_t* __restrict__ lbw,
    uint64_t* __restrict__ lbw_tail) {
  // (only the staged tile: 16 KiB a block keeps fs_rows at full occupancy;
  // a frame-start array beside it cost the var-size GET 3x in fs_rows)
  __shared__ __attribute__((aligned(16))) uint8_t stage[4][FT_STAGE];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t t = (int64_t)blockIdx.x * 4 + wv;
  const int64_t n = stream_len(n_dev, n_cap);
  if (t == 0) {
    // fs_link's minima and broken-link count, for the next scan; and its
    // barrier words (the big repair): every fs_link workgroup has ended
    // (stream order), so a late one of an abandoned barrier can no longer
    // leave an arrival or the abort flag to the next scan
    if (lane == 0) {
      lbw_tail[LW_MINS] = 0;
      lbw_tail[LW_MINS + 1] = 0;
      lbw_tail[LW_NOSPEC] = 0;
      lbw_tail[LW_GRID + FL_NB] = 0;
    }
    if (lane < LW_END - LW_BIG) lbw_tail[LW_BIG + lane] = 0;
  }
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

// A stream of one tile at most (handshakes, a SET_WATCHES frame, small
// batches): staged once and walked frame by frame by one wave — one launch
// instead of fs_tile, fs_link and fs_rows (the storm's two handshake
// streams a step were six launches).  Same results as the tiled scan.
__global__ __launch_bounds__(64) void fs_small(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ n_dev,
    int64_t n_cap, int64_t maxp, int64_t* __restrict__ foff,
    int32_t* __restrict__ flen, int64_t cap, int64_t* __restrict__ result) {
  __shared__ __attribute__((aligned(16))) uint8_t sb[FT_STAGE];
  const int lane = threadIdx.x;
  const int64_t n = stream_len(n_dev, n_cap);       // (<= FT_S)
  fc_stage<FT_S>(buf, n, 0, sb, lane);
  int32_t c = 0, k = 0;
  bool bad = false;
  const int32_t n32 = (int32_t)n;
  while (c + 4 <= n32) {
    const int32_t len = __builtin_amdgcn_readfirstlane(lds_be32(sb, c));
    if (len < 0 || (int64_t)len > maxp) { bad = true; break; }
    if (c + 4 + len > n32) break;                   // the carry
    if (lane == 0 && k < cap) {
      foff[k] = c + 4;
      flen[k] = len;
    }
    ++k;
    c += 4 + len;
  }
  if (lane == 0) {
    result[0] = k;
    result[1] = c;
    result[2] = bad ? 1 : 0;
    result[3] = k > cap ? 1 : 0;
  }
}

// ZKMI_FS_SMALL=0: one-tile streams take the tiled scan too (A/B)
static bool fs_small_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ZKMI_FS_SMALL");
    v = (e ? atoi(e) : 1) ? 1 : 0;
  }
  return v != 0;
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
  // X flags (2 per tile), then the words LW_* name
  p.off_lbw = take((size_t)(2 * tiles + LW_END) * 8);
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

// A block re-walks its own broken links before its ticket when it found
// more than this many (ZKMI_FL_LOCAL_MIN overrides FL_LOCAL_MIN, for A/B)
static int32_t fl_local_min() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ZKMI_FL_LOCAL_MIN");
    v = e ? atoi(e) : FL_LOCAL_MIN;
  }
  return v;
}

// fs_link's switches: bit 0 the exact chase before the rounds
// (ZKMI_FL_CHASE_FIRST=0 turns it off, for A/B)
static int32_t fl_flags() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ZKMI_FL_CHASE_FIRST");
    v = (e ? atoi(e) : 1) ? 1 : 0;
  }
  return v;
}

// fs_link's grid: the check's workgroups (the last to finish goes on).
static unsigned fl_blocks() { return 16; }

// The smallest plausible frame body of the tile map's nodes (the smallest
// ZooKeeper body is 8 bytes: a ping's xid + type).  A real frame that short
// is still framed exactly (the map sends its chain to the serial walk).
static int32_t fs_minb() { return 8; }

// scan flag: frames may be longer than the window (fs_tile's frontier
// passes past the window, and survivor exits past it as candidates)
constexpr int32_t FS_LONG = 2;

// `window` values with this bit: FS_LONG (zkmi.ops.batch.frame_window sets
// it when the window is below the stream's largest frame)
constexpr int32_t FS_WIN_LONG = 1 << 16;

static int fs_tpb() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ZKMI_FS_TPB");
    const int x = e ? atoi(e) : 4;
    v = (x == 1 || x == 2) ? x : 4;
  }
  return v;
}

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
    // a row per tile (fs_tile) + fs_link's: its phase clock, every block's
    // entry / check-done clocks, the common path's ticket / end clocks
    if (hipMalloc(&g_dbg, (tiles + FL_DBG_ROWS) * 8 * 8) != hipSuccess)
      return nullptr;
    (void)hipMemset(g_dbg, 0, (tiles + FL_DBG_ROWS) * 8 * 8);
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
// correctness (fs_tile / fs_link check every speculated entry).
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
  if (n_cap <= FT_S && !(flags & (1 | 0xFFFF00)) && fs_small_on() &&
      fs_dbg_buf(tiles) == nullptr) {
    fs_small<<<1, 64, 0, st>>>(buf, n_dev, n_cap, maxp, foff, flen, cap,
                               result);
    ZK_LAUNCH_CHECK();
    return 0;
  }
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
  uint64_t* mins = lbw + 2 * tiles + LW_MINS;
  int64_t* lastk = (int64_t*)(lbw + 2 * tiles + LW_LAST);
  unsigned long long* grid = (unsigned long long*)(lbw + 2 * tiles + LW_GRID);
  // X flags, the stats, the check's minima and fs_link's grid words start
  // at zero
  if (!clean &&
      hipMemsetAsync(lbw, 0, (size_t)(2 * tiles + LW_END) * 8, st) !=
          hipSuccess)
    return -4;
  int64_t* dbg = fs_dbg_buf(tiles);
  // tiles (waves) per block: four 12 KiB slices, 3 blocks a CU (as many
  // waves as two-slice blocks, half the workgroups to dispatch: GET 0.585
  // -> 0.581 ms, mix and watch -0.7 %, profiles/r5_fs_tpb_ab.log).  (One
  // 23 ms watch step seen once in a full-suite process was a host pause
  // between the test's event records — the collector — not K1: six full
  // and isolated runs since, either width, show none.)  ZKMI_FS_TPB = 1 /
  // 2 / 4 for A/B runs.
  const int tpb = fs_tpb();
  // tiles a wave: groups (the map once, the chain walked on) for streams
  // of large frames within a small window; tests of the link repair and
  // long-frame streams take single tiles
  int G = ((flags >> 4) & 15) + 1;
  if ((flags & (FS_LONG | 1 | 0xFFFF00)) || W > 512) G = 1;
  G = G >= 16 ? 16 : G >= 8 ? 8 : G >= 4 ? 4 : G >= 2 ? 2 : 1;
  const int64_t waves = (tiles + G - 1) / G;
  const unsigned tblocks = (unsigned)((waves + tpb - 1) / tpb);
#define ZK_FS_TILE(WW, LL)                                                   \
  fs_tile<WW, LL, 1><<<tblocks, 64 * tpb, FT_LDS * tpb, st>>>(               \
      buf, n_dev, n_cap, maxp, list, pre, sx, lbw, rent, rexit, rmeta, rcnt, \
      tiles, dbg, fs_minb(), flags, cx)
#define ZK_FS_GROUP(WW, GG)                                                  \
  fs_tile<WW, false, GG><<<tblocks, 64 * tpb, FT_LDS * tpb, st>>>(           \
      buf, n_dev, n_cap, maxp, list, pre, sx, lbw, rent, rexit, rmeta, rcnt, \
      tiles, dbg, fs_minb(), flags, cx)
  if (G == 16) {
    if (W == 256) ZK_FS_GROUP(256, 16);
    else ZK_FS_GROUP(512, 16);
  } else if (G == 8) {
    if (W == 256) ZK_FS_GROUP(256, 8);
    else ZK_FS_GROUP(512, 8);
  } else if (G == 4) {
    if (W == 256) ZK_FS_GROUP(256, 4);
    else ZK_FS_GROUP(512, 4);
  } else if (G == 2) {
    if (W == 256) ZK_FS_GROUP(256, 2);
    else ZK_FS_GROUP(512, 2);
  } else if (flags & FS_LONG) {
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
#undef ZK_FS_GROUP
  ZK_LAUNCH_CHECK();
  fs_link<<<fl_blocks(), FL_T, 0, st>>>(buf, n_dev, n_cap, maxp, sx, list, rcnt,
                                 pre, rent, rexit, rmeta, base, cap, result,
                                 lbw + 2 * tiles, blist, bsum, mins, lastk,
                                 grid, lbw, cx, dbg ? dbg + 8 * tiles : nullptr,
                                 fl_local_min(), fl_flags());
  ZK_LAUNCH_CHECK();
  fs_rows<<<(unsigned)((tiles + 3) / 4), 256, 0, st>>>(
      buf, n_dev, n_cap, list, pre, rmeta, rent, rexit, base, bsum, lastk,
      foff, flen, cap, lbw, lbw + 2 * tiles);
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

// rows = tiles + FL_DBG_ROWS: past the tiles' rows, fs_link's phase clock of
// a chase repair (start, chases done, barrier, links checked, end; [6] / [7]
// the exact chase's start and end), then every block's entry and check-done
// clocks (4 rows), then the common path's bases start / end ([0] / [1])
int zk_frame_scan_dbg(int64_t* host, int64_t tiles) {
  if (!zk::g_dbg || tiles > zk::g_dbg_tiles + zk::FL_DBG_ROWS) return -1;
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

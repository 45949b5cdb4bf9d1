// Internal declarations shared by the HIP translation units of liblpa_hip.so.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <string>

#include "../../include/lpa.h"

namespace lpa {

typedef unsigned long long u64;
typedef uint32_t u32;
typedef int32_t v4i __attribute__((ext_vector_type(4)));  // native 16-B vector (nontemporal-capable)

// ---------------------------------------------------------------------------
// Degree bins (SURVEY.md §7 kernel inventory).  Vertices of a rank's slice are
// sorted by degree (descending), so every bin is one contiguous range.
// ---------------------------------------------------------------------------
//   seg  deg > 1024         wave per 512-arc unit, staged     (k_lpa_units + hub combine)
//   w16/w8/w4/w2  deg <= 1024/512/256/128   wave per vertex, NC chunks (k_lpa_wave<NC>)
//   g64 .. g1 deg <= G          G lanes per vertex                (k_lpa_group<G>)
enum Bin { BIN_SEG = 0, BIN_W16 = 1, BIN_W8 = 2, BIN_W4 = 3, BIN_W2 = 4, BIN_G64 = 5, BIN_G32 = 6,
           BIN_G16 = 7, BIN_G8 = 8, BIN_G4 = 9, BIN_G2 = 10, BIN_G1 = 11, BIN_ISO = 12 };
static_assert(BIN_ISO + 1 == LPA_NBINS, "bin table");
// fcnt[] slots (per parity, 16): [b] the dirty-row count of bin b, [kFcntUnits] the unit
// list's, [kFcntSettled] set by a giant superstep's row settle (lpa_iter.hip)
// supersteps after L0 that are label-dense: their hub combine runs forked over two
// streams (launch_hub_combine) and the hub rows of <= kBlockMaxDeg2 arcs are tallied by
// k_lpa_block (block mode); from kDenseSupersteps + 2 on a superstep is "converged"
// (captured graphs, frontier lists)
constexpr int kDenseSupersteps = 2;
constexpr int kFcntUnits = LPA_NBINS;
constexpr int kFcntSettled = LPA_NBINS + 1;
static_assert(kFcntSettled < 16, "fcnt: 16 slots per parity");
// upper degree bound of each bin (bin b holds bin_max[b+1] < deg <= bin_max[b])
constexpr int kBinMaxDeg[LPA_NBINS] = {1 << 30, 1024, 512, 256, 128, 64, 32, 16, 8, 4, 2, 1, 0};

constexpr int kWaveMaxDeg = 512;      // wave-per-vertex LDS hash for 64 < deg <= 512
constexpr int kWideMaxDeg = 1024;     // ... and (w16, 16 chunks, 2048-slot table) up to 1024
constexpr int kSegArcs = 512;         // arcs per unit of a seg-bin row (one wave)
constexpr int kBlockMaxDeg = 4096;    // seg rows up to this degree: k_lpa_block in the label-dense supersteps
constexpr int kBlockMaxDeg2 = 8192;   // ... and up to this one: its 16-wave, 16K-slot form (one block per CU)
constexpr int kTallyKernels = 13;                  // stats kernels 0..12: the tally
constexpr int kTallyEv = 2 * kTallyKernels;        // events bracketing each tally kernel
// + join, after exchange, after scatter, after rebuild, lists start, lists end,
// k_lpa_block start, end
constexpr int kBinEvents = kTallyEv + 8;
static_assert(LPA_NKERNELS == kTallyKernels + 4, "stats: tally kernels + refresh, rebuild, lists, block");
constexpr uint32_t kFlagNoLocality = 0x100u;  // internal create flag (not in lpa.h)
// internal create flag: every device array of the handle comes from the stream-ordered
// pool on the creator's stream (the outlier stage's per-call L2 sub-graph: its memory is
// reused from call to call instead of hipMalloc / hipFree, which synchronise the device)
constexpr uint32_t kFlagPooled = 0x200u;
constexpr int kCombWords = 2048;      // expected staged words per combine bucket
constexpr int kCombSlots = 8192;      // LDS table slots of a combine block
constexpr int kCombDirect = 6144;     // <= this many staged words: one block, no buckets
constexpr int kMaxBucketsLg = 12;     // at most 4096 buckets per hub
constexpr int kMaxBuckets = 1 << kMaxBucketsLg;
constexpr int kChunkPos = 256;        // arc positions per scatter chunk of a changed vertex
// replicated-label refresh: scatter the changed vertices' labels while they touch at
// most this fraction of the arcs, otherwise rebuild al[] with one gather pass
constexpr double kRebuildFrac = 0.25;
// the al[] scatter marks dirty rows while <= this fraction of the arcs changed; above
// it the next superstep tallies every row
constexpr double kFrontierFrac = 0.005;
// superstep 1's column-run tiles (lpa_iter.hip k_first_runs): arcs per wave tile, 16 per
// lane; the row-start bitmap holds whole tiles plus the next tile's first word
constexpr int kRunTile = 1024;
// P = 1 label vectors of at least this many slots take the LDS hot-set rebuild
// (k_al_rebuild_hot); smaller ones stay in L2 / the Infinity Cache (k_al_rebuild_small)
constexpr int64_t kHotMinSlots = 4ll << 20;
// column class of the class-blocked rebuild: the 4-KB chunk (1024 slots) of the column's
// label, mod ncls.  (Line-interleaved classes, (c >> 5) & 7, fixed address bits 7-9 of an
// XCD's gathers and crowded them onto a few L2 channels: 2.5x fewer bytes fetched than
// the plain stream, yet 1.5x its time.)
// (ncls = 8 x phases classes: block group x streams classes x, x + 8, ... one phase after
// another, so an XCD's gathers cover 1 / ncls of the label vector at a time)
constexpr int kMaxBlkClasses = 32;
__host__ __device__ inline uint32_t col_class(int32_t c, uint32_t ncls) { return ((uint32_t)c >> 10) & (ncls - 1u); }

struct Segment {   // one unit of a seg-bin row
  int64_t begin;  // first arc (local CSR index)
  int32_t len;    // arcs in the unit (<= kSegArcs) | (index of the unit within its row << 10)
  int32_t v;      // local row (slot) index
};

// thread-local last error
void set_error(const char* fmt, ...);

#define LPA_HIP(call)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (call);                                                                \
    if (e_ != hipSuccess) {                                                                \
      ::lpa::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                       __LINE__);                                                          \
      return LPA_EHIP;                                                                     \
    }                                                                                      \
  } while (0)

#define LPA_TRY(call)        \
  do {                       \
    int rc_ = (call);        \
    if (rc_ != LPA_OK) return rc_; \
  } while (0)

// ---------------------------------------------------------------------------
// Device memory held by a handle.
// ---------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct Loopback;  // in-process collective over P handles on one device (lpa_comm.cpp)

// Bump arena a handle keeps for the outlier stage's L2 sub-graph (round 6): every device
// array of that per-call handle, scratch included, is carved from blocks the parent
// keeps from call to call, so a call issues no hipMallocAsync / hipFreeAsync for them
// (126 hipFreeAsync per L2 call at C3 blocked the host for 12.6 ms, one of them 4 ms).
// Reset by each L2 build; released with the parent.
struct Arena {
  struct Block {
    char* p;
    size_t bytes;
  };
  Block blocks[32] = {};
  int nblocks = 0;
  int cur = 0;       // block being carved
  size_t off = 0;    // offset in it
};

}  // namespace lpa

struct lpa_graph {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  // concurrent tally bins (0: wave bins, 1: row/group bins) and the hub combine's
  // bucket path (2); 4 streams = the 4 hardware queues of a process
  hipStream_t aux_stream[3] = {nullptr, nullptr, nullptr};
  hipEvent_t ev_fork = nullptr, ev_join[2] = {nullptr, nullptr};
  hipEvent_t ev_fork2 = nullptr, ev_join2[3] = {nullptr, nullptr, nullptr};  // hub combine tail, block tiers
  int32_t rank = 0, nranks = 1;
  // label-exchange collective backend (P > 1): RCCL communicator (one process per
  // GPU) or the in-process loopback group (P handles on one device, one host thread
  // each); neither = the caller-driven exchange (lpa_exchange_get/put)
  ncclComm_t comm = nullptr;
  lpa::Loopback* loop = nullptr;
  // host-staged collective (lpa_graph_create_hostcoll): each allgather is handed to the
  // caller's host function (MPI, torch.distributed gloo, a Spark barrier stage ...),
  // staged through a pinned host buffer (hc_buf: send + nranks * recv bytes, grown on use)
  lpa_allgather_fn hc_fn = nullptr;
  void* hc_ctx = nullptr;
  void* hc_buf = nullptr;
  size_t hc_bytes = 0;
  int64_t n_host_allgathers = 0;               // allgathers served by hc_fn (lpa_graph_info)
  hipEvent_t loop_ev[2] = {nullptr, nullptr};  // loopback: send-ready / copies-done marks
  int64_t n_exch_full = 0, n_exch_delta = 0;   // exchanges by mode (lpa_graph_info)
  int64_t n_graph_replays = 0;                 // supersteps replayed from a captured graph

  int64_t V = 0, m = 0;
  int64_t slice = 0;      // vertex slots per rank (P > 1: a power of two, lpa_build)
  int pow2_slices = 1;    // LPA_POW2_SLICES=0: tight slices (ceil(V / P) rounded to 64)
  int fused_bins = 1;     // LPA_FUSED_BINS: converged supersteps' bins in one launch per stream
                          // (0: a launch per bin, 2: the wave bins keep theirs)
  int units_pure = 1;     // LPA_UNITS_PURE=0: superstep 4 re-tallies every hub unit
  int keep_bits = 1;      // LPA_KEEP_BITS=0: superstep 3's scatter drops the arc giant bits
  int conv_streams = 2;   // LPA_CONV_STREAMS: streams of a converged superstep's tally (1-3)
  int64_t vpad = 0;       // nranks * slice
  int64_t own_begin = 0;  // rank * slice
  int64_t n_own = 0;      // real (non-padding) vertices owned
  int64_t arcs = 0;       // local arcs
  int32_t max_degree = 0;

  // CSR of the owned slice, internal (degree-ranked) numbering
  int64_t* rp = nullptr;    // [slice + 1]
  int32_t* col = nullptr;   // [arcs] global internal ids
  int32_t* new_of = nullptr;  // [V] dense id -> internal slot
  int32_t* old_of = nullptr;  // [vpad] internal slot -> dense id (-1 padding)
  int32_t* deg = nullptr;     // [V] symmetrised degree by dense id
  int32_t* lab[2] = {nullptr, nullptr};  // [vpad] ping-pong label vectors (replicated)
  int cur = 0;                // index of the current label vector
  int par = 0;                // superstep parity: which counter / queue-count set is live
  int64_t since_reset = 0;    // supersteps run since the labels were last L0

  // degree bins over the owned slice
  int64_t bin_begin[LPA_NBINS + 1] = {0};
  int64_t bin_arcs[LPA_NBINS] = {0};

  // hub path: rows longer than one segment.  Their segment tallies are staged
  // as tally words in stage[rp[h] .. rp[h] + wcount[h]) and merged by the hub
  // combine (lpa_hub.hip): small runs in a wave, mid-size runs in a block, large
  // runs partitioned into label-hash buckets (scat[], same layout as stage[]).
  lpa::Segment* segs = nullptr;
  int64_t n_segs = 0;
  int64_t n_hub = 0;              // rows with > kWideMaxDeg arcs (= the seg bin)
  lpa::u64* stage = nullptr;      // [hub arcs] staged unit tally words (unit j of row h:
                                  //  stage[rp[h] + j*kSegArcs ...), ucnt[hub_uoff[h] + j] words)
  int64_t* hub_uoff = nullptr;    // [n_hub + 1] first unit of each row (units = segs[])
  int32_t* ucnt = nullptr;        // [n_segs] staged words of each unit
  uint32_t* ugc = nullptr;        // [n_segs] superstep 2: the unit's giant-label votes ...
  uint32_t* umx = nullptr;        // [n_segs] ... and its fullest other-label bucket (k_lpa_units_giant)
  int32_t* ulist2 = nullptr;      // [n_segs] units of the rows k_hub_decide could not settle
  int32_t* gdec = nullptr;        // [4] their count, a constant 0 (the list-mode "fr_all"), the count of glist
  int32_t* glist = nullptr;       // [n_hub] block-tier rows k_hub_decide could not settle (k_lpa_block's list)
  lpa::u64* scat = nullptr;       // [hub arcs] bucket-partitioned words
  int32_t* hub_wcount = nullptr;  // [n_hub] staged words of a queued row (0 otherwise)
  lpa::u64* hub_best = nullptr;   // [n_hub] reduced tally word (bucketed hubs)
  int64_t* hub_hoff = nullptr;    // [n_hub + 1] first bucket counter of each hub
  int32_t* ghist = nullptr;       // [n_hub_buckets] words per bucket
  int32_t* gcur = nullptr;        // [n_hub_buckets] bucket offsets / scatter cursors
  int32_t* hub_lists = nullptr;   // [6 n_hub] queued rows: mid (T <= 1024), bucketed, wave path,
                                  //   mid (T <= 2048), mid (T <= 6144), small (list S)
  uint32_t* hub_tickets = nullptr; // fused hub kernels' last-block tickets (lpa_hub.hip)
  int32_t* hub_lcnt = nullptr;    // [2][8] per parity, queue lengths: mid1, bucketed, bucket items,
                                  //   chunk items, wave path, mid2, mid3, small (list S)
  int64_t hub_lane_begin = 0;     // rows [hub_lane_begin, n_hub) have <= 8 units
  int64_t hub_block2_begin = 0;   // rows [hub_block2_begin, hub_lane_begin) have <= 16 units (wide block tier)
  int first_runs = 1;             // LPA_FIRST_RUNS=0: superstep 1 by the hash tallies, not column runs
  bool cols_sorted = true;        // columns ascending inside each row (false: row-only sorted build)
  lpa::u64* first_best = nullptr; // [slice] superstep-1 best run word of rows spanning run tiles
  lpa::u64* rstart = nullptr;     // [arcs / 64 + pad] bit i: arc position i starts a row (crow[i] !=
                                  //   crow[i - 1]); k_first_runs reads it instead of crow (1 bit/arc)
  int64_t unit_lane_begin = 0;    // hub_uoff[hub_lane_begin]
  int64_t unit_block2_begin = 0;  // hub_uoff[hub_block2_begin]
  bool force_all_next = false;    // the next superstep tallies every row (after block mode)
  lpa::u64* items_cb = nullptr;   // [n_hub_buckets] (hub << 32 | bucket)
  lpa::u64* items_cc = nullptr;   // [n_hub_chunks]  (hub << 32 | 8-unit chunk)
  int64_t n_hub_buckets = 0, n_hub_chunks = 0;
  int32_t* dev_err = nullptr;     // [1] kernel-side error flags (checked after a call)

  // frontier (exact active set): a row whose neighbours all kept their label keeps
  // its own, L_{t+1}[v] = mode(L_t[N(v)]) = mode(L_{t-1}[N(v)]) = L_t[v], so only rows
  // with a changed neighbour are re-tallied.  The al[] scatter of superstep t marks
  // the rows (and hub units) whose al entries it rewrote in rdirty/udirty[par ^ 1];
  // k_frontier_lists turns them into per-bin row lists and a unit list at the start
  // of superstep t + 1 (clearing the flags), and the bin kernels walk only those.  fr_all[par] = 1:
  // every row is tallied (after L0, after an al[] rebuild, frontier off).  Skipped rows
  // need no write: the diff copies every changed label into the other label vector,
  // which is the next superstep's output (k_diff / k_delta_compact).
  int32_t* crow = nullptr;        // [arcs] row (local slot) of each arc position
  uint8_t* rdirty[2] = {nullptr, nullptr};  // [slice] per parity
  uint8_t* udirty[2] = {nullptr, nullptr};  // [n_segs] per parity (hub units)
  int32_t* fr_all = nullptr;      // [2] per parity: 1 = tally every row
  int32_t* flist = nullptr;       // [slice] dirty rows of this superstep, bin b at bin_begin[b]
  int32_t* ulist = nullptr;       // [n_segs] dirty hub units of this superstep
  int32_t* fcnt = nullptr;        // [2][16] per parity: list lengths (bins 0..12, units at 13)
  int frontier = 1;               // LPA_FRONTIER / lpa_set_frontier

  // replicated neighbour labels (GraphX ReplicatedVertexView analogue):
  // al[i] = L_cur[col[i]]; kept current by scatter (few changes) or rebuild
  int32_t* al = nullptr;        // [arcs]
  // al0[i] = L0[col[i]] (label-independent: the dense id of the column), kept when
  // superstep 1 runs by column runs.  A reset then leaves al stale (al_pending): the
  // column-run superstep reads al0 and its refresh rebuilds al, or fills it from al0
  // when it only scatters; any other first use copies al0 first (ensure_al).
  int32_t* al0 = nullptr;       // [arcs] or nullptr
  bool al_pending = false;
  bool al_is_l0 = false;        // al holds L0[col] already (the L2 sub-graph's build writes it)
  uint32_t* gbits = nullptr;    // [vpad / 32] rebuild: bit u = (L[u] == G), the giant label
  int32_t* gword = nullptr;     // [8] G of the last refreshed vector (k_giant_pick), worth-trying flag,
                                //     abits valid (bits-mode rebuild, no scatter since), [3] hot-slot
                                //     giant-bit count (k_giant_bits), [4] superstep 4 bins: 0 = lists,
                                //     [5] giant-code refresh taken (superstep 2 settles from al2),
                                //     [6] superstep 2's wave bins: 0 = lists of the unsettled rows,
                                //     [7] superstep 3's row bins (code refresh), [9] superstep 4's
                                //     k_abits_pass ran (its bits valid for the rows below the hubs),
                                //     [10] / [11] superstep 4's impure-unit list mode / count
                                //     (k_units_pure); 16 words
  // giant codes (round 5, lpa_iter.hip "Giant codes"): the refresh after superstep 1 (or
  // 2), when one label G carries the hubs but not half the hot slots (R-MAT), writes a
  // 2-bit code per arc instead of al[] (code 0 = G, else 1 + a label hash mod 3; 16 arcs
  // to a word of al2) for the rows above the cut (code_lbin), and al[] only for the
  // positions of the rows below it.  Round 6: every rank of a partitioned job too (G is
  // picked from the replicated vector, the same on every rank; each rank codes its own arcs)
  bool code_ok = false;         // the handle can take that refresh (the LDS hot-set rebuild:
                                //   P = 1, or P > 1 with power-of-two slices, rebuild_ranked)
  uint32_t* code2 = nullptr;    // [vpad / 16] 2-bit code of every slot's label (16 per word)
  uint32_t* al2 = nullptr;      // [(code_pcut rounded up to 512 + 512) / 16] 2-bit code of every
                                //   arc's column label (arc i: word i / 16, bits 2 (i % 16))
  bool gather = false;          // gather mode: supersteps 1..kGatherSteps tally from L[col[i]] with
                                //   no al[] refresh; the last of them rebuilds al (lpa_build)
  int32_t code_lbin = lpa::BIN_G8;   // first bin whose rows keep their labels in a code refresh
                                //   (lpa_build: g64 when the label vector is <= 64 MB, else g8;
                                //   LPA_CODE_LBIN=5|8 forces either, for tests)
  int32_t code_lbin_env = -1;   // LPA_CODE_LBIN at create time (-1: by size)
  int codes_env = 1;            // LPA_GIANT_CODES=0: no giant-code refresh (A/B, tests)
  int64_t code_pcut = 0;        // its first arc position
  bool code3 = false;           // superstep 3 follows a giant-code refresh (read by the host
                                //   before it: its schedule differs, see run_supersteps)
  int32_t* h_flag = nullptr;    // [1] pinned host word for that read
  int32_t* h_err = nullptr;     // [1] pinned host copy of dev_err (read at the end of a call)
  unsigned long long* abits = nullptr;  // [arcs / 64] bit i = (al[i] == G): the bits-mode rebuild's by-product
  int64_t* cptr = nullptr;      // [vpad + 1] CSC: arcs of this rank whose column is u ...
  uint32_t* cpos = nullptr;     // [arcs]      ... are at positions cpos[cptr[u] .. cptr[u+1])
  // per-superstep change bookkeeping (device)
  // scatter chunks: column u's positions cpos[cptr[u] ..) in pieces of kChunkPos,
  // numbered statically: chunks cch[u] .. cch[u+1] - 1 belong to u (cowner[])
  int64_t n_chunks = 0;
  int64_t* cch = nullptr;       // [vpad + 1]
  int32_t* cowner = nullptr;    // [n_chunks]
  uint8_t* chflag = nullptr;    // [n_chunks, padded to 16] changed multi-chunk columns' flags
  int64_t n_chunk_scan = 0;     // chunks below this belong to every multi-chunk column
  int32_t* chlist = nullptr;    // [vpad] changed one-chunk columns (count: counters[par][0])
  int rebuild_hot = 1;                      // LDS hot-label rebuild (LPA_REBUILD_HOT=0 disables)
  // class-blocked labels-mode rebuild (P = 1, lpa_iter.hip rebuild_pieces): rows of
  // degree > block_deg keep their columns in (class, column) order (col_class); the
  // class segments cut into <= 64-arc pieces, listed per class
  // (padded to multiples of 8) so that one block group (one XCD) gathers one class
  int block_deg = 512;                      // LPA_BLOCK_DEG (0: off; a power of two)
  int64_t block_min_slots = 32ll << 20;     // ... on label vectors of >= this many slots
                                            //   (LPA_BLOCK_MIN_SLOTS): C5 176 -> 186 GTEPS,
                                            //   but C3 (64 MB of labels) 0.9 ms slower
  lpa::u64* blk_pieces = nullptr;           // [n] (len << 32 | first position)
  int blk_classes = 8;                      // 8 x phases (kMaxBlkClasses at most)
  int64_t blk_off[lpa::kMaxBlkClasses + 1] = {}; // class x: pieces [blk_off[x], blk_off[x + 1])
  int64_t blk_a0 = 0;                       // arcs [0, blk_a0) are listed (a multiple of 512)
  int64_t blk_rows = 0;                     // rows in (class, column) order
  int serial = 0;                           // LPA_SERIAL=1: all tally kernels on one stream (profiling)
  int use_graphs = 1;                       // LPA_GRAPHS=0: no captured superstep graphs
  // captured supersteps: [0, 4) converged per (cur, par); [4, 12) supersteps 2 and 3 per
  // (superstep, cur, par); [12, 16) superstep 3 after a giant-code refresh; [16, 24) the
  // converged supersteps of gather mode (5 and 6, cur, par)
  hipGraphExec_t gexec[24] = {};
  int locality = 2;                         // LPA_LOCALITY: neighbour keys of the locality order (0: plain)
  unsigned long long* counters = nullptr;  // [2][4] per parity: [0] chunk count, [1] dirty arcs

  // label exchange (P > 1, lpa_exchange.hip): changed-label deltas
  lpa::u64* dsend = nullptr;                 // [slice] this rank's (slot << 32 | label)
  lpa::u64* drecv = nullptr;                 // [nranks * dcap] gathered deltas
  unsigned long long* dcount = nullptr;      // [1 + nranks] own count, then every rank's (caller-driven)
  unsigned long long* h_dcounts = nullptr;   // [3 nranks] pinned host copy of the count triples
  // giant-compressed exchange (lpa_exchange.hip): the giant-label bitmap of every slice
  // ([nranks][slice / 64] words, own slice in place) and the changed non-G entries
  lpa::u64* gsend = nullptr;                 // [slice] this rank's changed non-G (slot << 32 | label)
  unsigned long long* gbm = nullptr;         // [nranks * slice / 64] bit = (label == G)
  unsigned long long* xpair = nullptr;       // [3 + 3 nranks] own (delta count, giant count, posted
                                             //   request), then every rank's
  int64_t n_exch_giant = 0;                  // exchanges done in the giant-compressed form
  int64_t dcap = 0;                          // delta entries per rank (slice / 4)
  int64_t last_exchange_delta = -1;          // entries per rank of the last exchange (-1 full)
  bool prev_delta_ok = false;                // the last exchange was a delta: the two label
                                             //   buffers agree outside the own slice
  int64_t post_cap = 0;                      // posted delta capacity of the next exchange (0: none),
                                             //   agreed over the ranks from the gathered triples
  int64_t post_fixed = -1;                   // lpa_set_posted: this rank's request, -1 adaptive, 0 off,
                                             //   > 0 fixed (the smallest capacity requested wins)
  int64_t n_exch_posted = 0;                 // delta exchanges that went out before the count read
  int64_t n_exch_post_missed = 0;            // posted exchanges whose counts exceeded the capacity
  hipEvent_t cnt_ev = nullptr;               // the count pairs reached h_dcounts

  // original edge list kept for the outlier stage (device, dense ids)
  int32_t* e_src = nullptr;
  int32_t* e_dst = nullptr;
  // its distinct directed edges (s << 32 | d), sorted: built by the first outlier call
  // and kept (label-independent topology, as GraphFrames' cachedTopologyGraphX)
  lpa::u64* de_keys = nullptr;
  int64_t de_n = -1;                        // -1: not built yet
  // ... and, for the L2 sub-graph build (first L2 call, kept): the same edges in (d, s)
  // order as (d << 32 | index into de_keys), their s, and the first index of every
  // vertex's run in either order ([V + 1] each)
  lpa::u64* de_t = nullptr;
  uint32_t* de_ts = nullptr;
  int64_t* de_out_off = nullptr;
  int64_t* de_in_off = nullptr;
  void* host_pin = nullptr;                 // outlier stage: pinned staging of host labels in /
  size_t host_pin_bytes = 0;                //   arrays out (kept with the handle)

  int64_t device_bytes = 0;
  bool pooled = false;                      // kFlagPooled: arrays from the stream-ordered pool
  lpa::Arena* arena = nullptr;              // this handle's arena for its L2 sub-graphs (lazy)
  lpa_graph* arena_from = nullptr;          // a pooled L2 sub-graph: allocate from this parent's arena
  bool no_scatter = false;                  // no CSC position index: every refresh rebuilds al[]
                                            //   (the outlier stage's 5-superstep L2 sub-graph)
  bool borrowed = false;                    // aux streams / fork-join events belong to a parent handle
  hipEvent_t ev[2 * LPA_STATS_MAX_ITERS + 2] = {};
  hipEvent_t bin_ev[LPA_STATS_MAX_ITERS * lpa::kBinEvents] = {};
};

namespace lpa {

// allocation helpers (track bytes on the handle)
int dev_alloc(lpa_graph* g, void** p, size_t bytes);
// stream-ordered temporaries (lpa_prims.hip); tmp_trim returns the pool's cached
// memory to the device
int tmp_alloc(void** p, size_t bytes, hipStream_t s);
void tmp_free(void* p, hipStream_t s);
void tmp_trim(int device);
void dev_free(lpa_graph* g, void* p);
// build temporaries: like dev_alloc / dev_free without the accounting (both draw on the
// stream-ordered pool for a pooled handle)
int scratch_alloc(lpa_graph* g, void** p, size_t bytes);
void scratch_free(lpa_graph* g, void* p);

// primitives (lpa_prims.hip)
// LSD radix sort of u64 keys in place (tmp: same length); sorts digits at the
// given bit shifts (8-bit digits), in order.  Result ends in `keys`.
int radix_sort_u64(u64* keys, u64* tmp, int64_t n, const int* shifts, int nshifts,
                   hipStream_t s);
// exclusive scan of int32 input into int64 output (n + 1 entries: out[n] = total)
int exclusive_scan_i32_i64(const int32_t* in, int64_t* out, int64_t n, hipStream_t s);
int exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t s);
// exclusive scan of 0/1 bytes into uint32 positions (n + 1 entries; the total < 2^32)
int exclusive_scan_u8_u32(const uint8_t* in, uint32_t* out, int64_t n, hipStream_t s);
int bits_for(uint64_t maxval);  // bits needed to represent maxval (0 -> 0)

// build (lpa_build.hip)
int build_graph(lpa_graph* g, const int32_t* src, const int32_t* dst, int64_t m, int32_t V,
                uint32_t flags);
int init_labels(lpa_graph* g);
// the outlier stage's L2 sub-graph (P = 1, pooled handle g, V vertices) straight from the
// parent's sorted distinct edge orders: E' = distinct (s, d) with L[s] == L[d], no sort
// of arcs (lpa_build.hip)
// mo (nullable): the intra marks of the parent's (s, d)-ordered distinct edges, when the
// caller's incident-edge pass already computed them (k_incident<true>)
int build_graph_l2(lpa_graph* g, const lpa_graph* parent, const int32_t* L, const uint8_t* mo);
int build_hub_tables(lpa_graph* g, const int32_t* deg_own);  // lpa_hub.hip
// join = false: the forked bucket path's end is recorded in ev_join2[0] and the caller
// joins it (main-stream work can be queued behind the mid tiers first)
int launch_hub_combine(lpa_graph* g, int32_t* Lown, bool fork, bool join = true,
                       bool giant = false);  // lpa_hub.hip
int launch_hub_decide(lpa_graph* g, int32_t* Lown, int64_t h_end, const int32_t* gsel);  // lpa_hub.hip
bool block_mode_now(const lpa_graph* g);  // lpa_iter.hip
bool fused_now(const lpa_graph* g);       // lpa_iter.hip
int64_t block_rows_begin(const lpa_graph* g);  // first row of the block tiers (lpa_iter.hip)
int rebuild_arc_labels(lpa_graph* g);  // al[i] = lab[cur][col[i]]
// the caller-driven full exchange (lpa_exchange_put) completes the superstep just run:
// its refresh rebuilds every arc label, and may take the giant codes as the in-library
// refresh of that superstep would
int refresh_after_put(lpa_graph* g);
// P > 1: the LDS hot-set rebuild's rank-strided form applies (power-of-two rank count and
// slice, each slice holding its share of the kHotRankedLabels hottest labels)
constexpr int kHotRankedLabels = 32768;
inline bool rebuild_ranked(const lpa_graph* g) {
  const auto pow2 = [](int64_t x) { return x > 0 && (x & (x - 1)) == 0; };
  return g->nranks > 1 && pow2(g->nranks) && pow2(g->slice) && g->nranks <= kHotRankedLabels &&
         g->slice >= kHotRankedLabels / g->nranks;
}
int ensure_al(lpa_graph* g);           // al valid (copies al0 after a lazy reset)
int frontier_all(lpa_graph* g, int par);  // next tally of parity `par` takes every row

// iteration (lpa_iter.hip)
// last_refresh = false: the last superstep leaves al[] stale (a handle whose labels are
// read and which is then destroyed: the outlier stage's L2 sub-graph)
int run_supersteps(lpa_graph* g, int32_t n, lpa_stats* st, bool last_refresh = true);
int gather_labels(lpa_graph* g, int32_t* out_dense_dev);

// collective backend (lpa_comm.cpp): allgather of `count` elements of `elem` bytes
// per rank in rank order (in place when send == recv + rank * count * elem),
// stream-ordered on s, on the handle's RCCL communicator or loopback group
inline bool has_collective(const lpa_graph* g) {
  return g->comm != nullptr || g->loop != nullptr || g->hc_fn != nullptr;
}
// the superstep has a label-exchange step: P > 1, or an RCCL communicator / host
// collective at any P (a one-rank job of the distributed path runs the same exchange
// code, its allgather of one rank included)
inline bool exchanges(const lpa_graph* g) { return g->nranks > 1 || g->comm != nullptr || g->hc_fn != nullptr; }
int coll_allgather(lpa_graph* g, const void* send, void* recv, size_t count, int elem, hipStream_t s);
int loopback_attach(lpa_graph* g, Loopback* lb);  // registers the handle's rank slot
int loopback_ranks(const Loopback* lb);
void loopback_detach(lpa_graph* g);

// label exchange (lpa_exchange.hip)
int exchange_alloc(lpa_graph* g);
void exchange_free(lpa_graph* g);
int exchange_compact(lpa_graph* g, const int32_t* Lc, const int32_t* Ln);
lpa::u64* exchange_recv_buf(lpa_graph* g);
unsigned long long* exchange_recv_counts(lpa_graph* g);
int exchange_finish_delta(lpa_graph* g, int32_t* Lc, int32_t* Ln, int64_t cap, int par,
                          const unsigned long long* counts, int cs, bool posted = false);
int exchange_collective(lpa_graph* g, const int32_t* Lc, int32_t* Ln, bool first, bool* changes_listed);
int launch_refresh_ext(lpa_graph* g, const int32_t* Lc, const int32_t* Ln, bool diff_done, int par);

// outlier (lpa_outlier.hip)
int outlier(lpa_graph* g, const int32_t* labels, int32_t labels_on_device, int32_t mode,
            int32_t sub_iter, int64_t* size_hist, int64_t* incident, int32_t* sub_labels,
            uint8_t* flags, lpa_outlier_summary* summary, int32_t out_on_device);
int quality(lpa_graph* g, const int32_t* labels, int32_t labels_on_device, lpa_quality_summary* out);

}  // namespace lpa

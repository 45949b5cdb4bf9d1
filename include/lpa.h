/*
 * lpa.h -- C ABI of the MI355X-native label-propagation + outlier library
 * (liblpa_hip.so, hand-written HIP for gfx950, RCCL for the multi-GPU label
 * exchange).  Plain pointers and sizes only; no torch types.
 *
 * Each entry point replaces one piece of the reference's hot path, which is
 * the JVM call chain behind
 *     /root/reference/CommunityDetection/Graphframes.py:78   GraphFrame(v, e)
 *     /root/reference/CommunityDetection/Graphframes.py:81   .labelPropagation(maxIter=5)
 *     /root/reference/CommunityDetection/Graphframes.py:92-137 outlier stage
 * (GraphFrames 0.6.0 / Spark 2.4.5 GraphX, not vendored; see SURVEY.md §2.2
 * U1-U5).  Semantics: SURVEY.md Appendix A (LPA-DET) and Appendix B
 * (OUTLIER-DET).  Bindings a host would add: INTEGRATION.md.
 *
 * Conventions
 *   - vertex ids are dense int32 in [0, V); the dense order is the ascending
 *     order of the caller's original ids, so "smallest label" is preserved;
 *   - every function returns LPA_OK (0) or a negative LPA_E* code; the
 *     message is available from lpa_last_error() (thread-local);
 *   - calls block until the device work they issued has finished;
 *   - a handle is not thread-safe; distinct handles are independent.
 */
#ifndef LPA_H_
#define LPA_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LPA_OK 0
#define LPA_EINVAL (-22)   /* bad argument (maxIter <= 0, id out of range, ...) */
#define LPA_ENOMEM (-12)   /* device or host allocation failed                  */
#define LPA_ENODEV (-19)   /* no HIP device / bad device ordinal                */
#define LPA_EHIP (-1000)   /* HIP runtime error                                  */
#define LPA_ERCCL (-2000)  /* RCCL error                                         */
#define LPA_EOVERFLOW (-75) /* kernel-side capacity overflow (hub combine table) */

/* lpa_graph_create* flags */
#define LPA_INPUT_DEVICE 0x1u /* src/dst are device pointers on `device`        */

#define LPA_NBINS 13   /* 0 seg 1 w16 2 w8 3 w4 4 w2 5 g64 6 g32 7 g16 8 g8 9 g4 10 g2 11 g1 12 isolated */
#define LPA_NKERNELS 17 /* timed: 0 seg 1 hub 2 w16 3 w8 4 w4 5 w2 6 g64 7 g32 8 g16 9 g8 10 g4 11 g2 12 g1
                          13 refresh (diff + al[] scatter) 14 al[] rebuild 15 frontier lists
                          16 block-per-row hub tally (label-dense supersteps) */
#define LPA_STATS_MAX_ITERS 64

typedef struct lpa_graph lpa_graph;

/* Per-call timing, filled by lpa_step / lpa_run (HIP events on the handle's stream).
 * iter_ms: always (events around each superstep; converged single-GPU supersteps
 * still replay their captured graph).  kernel_ms / exchange_ms: only on a handle in
 * the serialized profiling schedule (lpa_set_serial(g, 1)), where events bracket
 * every tally kernel so each time is that kernel's standalone duration. */
typedef struct lpa_stats {
  int32_t iters;                           /* supersteps executed by this call          */
  int32_t n_iter_ms;                       /* entries filled in iter_ms                 */
  float iter_ms[LPA_STATS_MAX_ITERS];      /* device time per superstep (incl. exchange) */
  float kernel_ms[LPA_NKERNELS];           /* summed device time per kernel (serial)    */
  float exchange_ms;                       /* summed label-exchange time (serial)       */
  double total_ms;                         /* device time of all supersteps of the call */
} lpa_stats;

/* Layout facts of a built graph (this rank's slice). */
typedef struct lpa_graph_info {
  int64_t V;            /* vertices (global)                                  */
  int64_t m;            /* input directed edges (global)                      */
  int64_t arcs;         /* symmetrised arcs owned by this rank (= 2m at P=1)  */
  int64_t slice;        /* vertex slots per rank (V padded to P * slice)      */
  int64_t own_begin;    /* first global (internal) vertex slot of this rank   */
  int32_t rank, nranks, device;
  int32_t max_degree;   /* global maximum symmetrised degree                  */
  int64_t bin_vertices[LPA_NBINS]; /* degree bins, see LPA_NBINS */
  int64_t bin_arcs[LPA_NBINS];
  int64_t hub_vertices; /* vertices split over several segments (global merge) */
  int64_t segments;     /* segment count of bin 0                             */
  int64_t device_bytes; /* device memory held by the handle                   */
  int64_t exchanges_full;  /* P > 1: label exchanges done as a full allgather   */
  int64_t exchanges_delta; /* P > 1: label exchanges done as changed-label deltas */
  int64_t exchanges_giant; /* P > 1: label exchanges done giant-compressed (bitmap of the
                              giant label + changed non-giant labels) */
  int64_t blocked_rows;    /* P = 1: rows whose columns are in (class, column) order for
                              the class-blocked al[] rebuild (0: off, LPA_BLOCK_DEG)  */
  int64_t blocked_pieces;  /* ... and the rebuild's piece-list length                */
  int64_t code_refresh;    /* 1: the last refresh took the giant codes (the next superstep
                              settles rows from 2-bit label codes; every
                              rank of a partitioned job since ABI 7) -- read after a
                              superstep-1 step; 0 otherwise (since ABI 6)              */
  int64_t graph_replays;   /* supersteps run by replaying a captured HIP graph (the
                              converged ones, P = 1 also supersteps 2-3; since ABI 6)  */
  int64_t exchanges_posted; /* P > 1: delta exchanges sent at a capacity fixed before the
                              count read, so the GPU works through it (since ABI 6)   */
  int64_t exchanges_post_missed; /* ... posted ones whose counts exceeded the posted
                              capacity: exchanged again in the form that fits          */
  int64_t gather_mode;     /* 1: the tallies read L[col[i]] and no al[] refresh runs (one
                              GPU, label vector <= 4 MB, no row above 128 arcs; since ABI 6) */
  int64_t host_allgathers; /* allgathers served by the host collective's function
                              (lpa_graph_create_hostcoll; since ABI 7)                 */
} lpa_graph_info;

/* Outlier summary. */
typedef struct lpa_outlier_summary {
  int64_t n_groups;      /* L1: distinct communities; L2: distinct (community, sub-label) groups */
  int64_t k;             /* L1: n_groups / 10                                        */
  int64_t threshold;     /* L1: size threshold (flag iff size < threshold)           */
  int64_t n_flagged;     /* vertices flagged                                         */
  int64_t n_communities; /* distinct top-level communities                           */
  int64_t n_communities_flagged; /* L2: communities with >= 1 flagged sub-community  */
  int64_t distinct_edges;        /* distinct directed (s,d) pairs                     */
} lpa_outlier_summary;

/*
 * Build the symmetrised, degree-sorted CSR of the multigraph (src[i], dst[i]),
 * i < m, on HIP device `device`.  Duplicate edges are kept (each is a vote),
 * a self-loop gives two votes (GraphX sendMessage both ways).
 * Replaces: GraphFrame.__init__ + cachedTopologyGraphX / GraphX Graph build
 * (Graphframes.py:78; U1, U2, U5 in SURVEY.md §2.2).
 */
int lpa_graph_create(const int32_t* src, const int32_t* dst, int64_t m, int32_t V,
                     int32_t device, uint32_t flags, lpa_graph** out);

/* RCCL unique id (128 bytes) for lpa_graph_create_dist; produced on one rank and
 * broadcast by the caller (MPI, torch.distributed, ...). */
int lpa_comm_unique_id(uint8_t id_out[128]);

/*
 * Multi-GPU build: one process per GPU.  Every rank passes the SAME edge list;
 * the rank keeps the CSR rows of its vertex slice (degree-ranked round-robin
 * 1D partition) and refreshes the replicated label vector with one RCCL
 * allgather per superstep.  Results are bit-identical to
 * the single-GPU build.  Replaces the Spark shuffle of aggregateMessages (U5).
 * comm_id == NULL with nranks > 1 selects the caller-driven exchange below.  A
 * comm_id with nranks == 1 builds a one-rank job of the same path (the exchange
 * step and its ncclAllGather run every superstep; labels as lpa_graph_create).
 */
int lpa_graph_create_dist(const int32_t* src, const int32_t* dst, int64_t m, int32_t V,
                          int32_t device, uint32_t flags, int32_t rank, int32_t nranks,
                          const uint8_t comm_id[128], lpa_graph** out);

/*
 * In-process loopback collective (SURVEY.md §8(e) "fake backend"): P handles on ONE
 * device, each created with lpa_graph_create_loopback and driven by its OWN host
 * thread (lpa_run / lpa_step concurrently, as P processes would).  The library's
 * exchange runs unchanged -- full/delta switch, host count read, in-place
 * allgather, delta chain -- with the allgather done as stream-ordered D2D copies
 * between the handles instead of ncclAllGather.  lpa_loopback_destroy on a group
 * that still has handles attached aborts it (their collectives fail) and leaves the
 * free to the last handle's lpa_graph_destroy.  lpa_loopback_abort releases every thread waiting in a collective
 * (each then fails with LPA_ERCCL); a rank whose peers never arrive fails the
 * same way after 300 s.
 */
/*
 * Host-staged collective (round 6): the same in-library exchange as the RCCL path --
 * full / delta / giant-compressed forms, the posted delta and its stand-down, the
 * per-rank count triple -- with every allgather handed to the caller's host function:
 *   allgather(send, recv, bytes_per_rank, ctx) gathers every rank's `bytes_per_rank`
 *   bytes from `send` into `recv` in rank order (nranks * bytes_per_rank bytes) and
 *   returns 0 (non-zero: the superstep fails with LPA_ERCCL).
 * Both buffers are pinned host memory owned by the library, valid during the call; the
 * function runs on the thread that called lpa_step / lpa_run, once per allgather, and
 * every rank calls it the same number of times with the same size.  For clusters
 * without RCCL between the ranks: MPI_Allgather, torch.distributed (gloo), a Spark
 * barrier stage moving the bytes through the driver.  PCIe-staged: the RCCL build
 * (lpa_graph_create_dist with a comm id) is the fast path between MI355X GPUs.
 */
typedef int (*lpa_allgather_fn)(const void* send, void* recv, int64_t bytes_per_rank, void* ctx);
int lpa_graph_create_hostcoll(const int32_t* src, const int32_t* dst, int64_t m, int32_t V,
                              int32_t device, uint32_t flags, int32_t rank, int32_t nranks,
                              lpa_allgather_fn allgather, void* ctx, lpa_graph** out);

typedef struct lpa_loopback lpa_loopback;
int lpa_loopback_create(int32_t nranks, lpa_loopback** out);
void lpa_loopback_abort(lpa_loopback* group);
void lpa_loopback_destroy(lpa_loopback* group);
int lpa_graph_create_loopback(const int32_t* src, const int32_t* dst, int64_t m, int32_t V,
                              int32_t device, uint32_t flags, int32_t rank, lpa_loopback* group,
                              lpa_graph** out);

/*
 * Caller-driven label exchange (a handle built by lpa_graph_create_dist with
 * nranks > 1 and comm_id == NULL performs no RCCL collective): after each
 * lpa_step(g, 1) the caller collects every rank's owned slice of the current
 * label vector (lpa_exchange_get: `slice` entries, internal slot order) and
 * writes the concatenation of all slices in rank order back to every rank
 * (lpa_exchange_put: nranks * slice entries).  Used to test the partitioned
 * path with P virtual ranks on one device (SURVEY.md §8(e) fake backend).
 * Host buffers.
 */
int lpa_exchange_get(lpa_graph* g, int32_t* slice_out);
int lpa_exchange_put(lpa_graph* g, const int32_t* full_in);
/*
 * Delta form of the caller-driven exchange (the protocol the in-library RCCL
 * exchange uses in converged supersteps, lpa_exchange.hip): after lpa_step(g, 1)
 * lpa_exchange_get_delta returns this rank's CHANGED owned labels as
 * (local slot << 32 | label) entries (entries_out: room for `slice` entries) and
 * their count; the caller lays every rank's entries out as [nranks][cap]
 * (cap >= every count, cap <= slice / 4) and passes them with the counts to
 * lpa_exchange_put_delta on every rank.  Host buffers.
 */
int lpa_exchange_get_delta(lpa_graph* g, uint64_t* entries_out, int64_t* count_out);
int lpa_exchange_put_delta(lpa_graph* g, const uint64_t* entries, const int64_t* counts, int64_t cap);

/* Profiling control: serial != 0 queues every tally kernel on the handle's main
 * stream (no concurrent bins), so per-kernel times in lpa_stats are standalone
 * durations.  Labels are identical either way. */
int lpa_set_serial(lpa_graph* g, int32_t serial);
/* Frontier (default on; LPA_FRONTIER=0 at create time turns it off): a superstep
 * re-tallies only the rows with a neighbour whose label changed in the previous
 * superstep -- exact, since a row whose neighbourhood labels are unchanged has the
 * same mode (GraphX Pregel's active-set idea applied to LPA).  Off: every row is
 * tallied every superstep.  Labels are identical either way. */
int lpa_set_frontier(lpa_graph* g, int32_t on);
/* P > 1 with a communicator or loopback group: capacity of the posted delta exchange
 * (converged supersteps after a delta exchange: the changed-label entries go out at a
 * capacity fixed before the per-rank counts are read, so the GPU works through the
 * host's read; a count above it makes the queued apply stand down and the host exchange
 * again in the form that fits).  cap < 0: adaptive (default: twice the last largest
 * count, 1024..131072 entries); 0: off (the host reads the counts first); > 0: that
 * fixed capacity (testing: 1 exercises the stand-down path).  The value is this rank's
 * REQUEST: it travels with the next per-rank count exchange and every rank posts the
 * smallest capacity requested by any rank (0 if any rank turned posting off), from the
 * superstep after that exchange on -- so ranks never disagree on the allgather size,
 * whichever ranks call this and when.  Labels are identical either way.  Since ABI 6. */
int lpa_set_posted(lpa_graph* g, int64_t cap);
/* Run on a caller-provided hipStream_t (NULL = the handle's own stream). */
int lpa_set_stream(lpa_graph* g, void* hip_stream);

/* Labels := L0 (every vertex its own id; LabelPropagation.run mapVertices(vid => vid)). */
int lpa_reset(lpa_graph* g);

/* Continue the synchronous BSP loop by n_supersteps (Pregel.apply iterations). */
int lpa_step(lpa_graph* g, int32_t n_supersteps, lpa_stats* stats /* nullable */);

/* Current labels indexed by dense vertex id; out is host memory unless out_is_device. */
int lpa_get_labels(lpa_graph* g, int32_t* labels_out, int32_t out_is_device);

/*
 * labelPropagation(maxIter): reset + max_iter supersteps + labels.
 * max_iter <= 0 -> LPA_EINVAL ("Maximum of steps must be greater than 0", U3 require).
 * Replaces: GraphFrame.labelPropagation -> lib.LabelPropagation.run ->
 * graphx.lib.LabelPropagation.run -> Pregel.apply (Graphframes.py:81).
 */
int lpa_run(lpa_graph* g, int32_t max_iter, int32_t* labels_out, int32_t out_is_device,
            lpa_stats* stats /* nullable */);

/*
 * Outlier stage over `labels` (dense-id indexed; host unless labels_on_device).
 * mode 1 = L1 (top-level community-size threshold), mode 2 = L2 (second LPA of
 * sub_iter supersteps on the intra-community distinct-edge subgraph, threshold
 * per community).  Outputs are host arrays of V entries, each nullable:
 *   size_hist[l]   members of community l              (Graphframes.py:100-104, :120)
 *   incident[l]    distinct directed edges touching l  (Graphframes.py:107-118)
 *   sub_labels[v]  L2 only: second-level label         (Graphframes.py:121-128)
 *   flags[v]       1 = outlier                          (Graphframes.py:130-137)
 * The first call on a handle builds its distinct directed edge set (topology) and a
 * pinned host staging area of 25 bytes per vertex for the host copies; both are kept
 * with the handle and released by lpa_graph_destroy.
 */
int lpa_outlier(lpa_graph* g, const int32_t* labels, int32_t labels_on_device, int32_t mode,
                int32_t sub_iter, int64_t* size_hist, int64_t* incident, int32_t* sub_labels,
                uint8_t* flags, lpa_outlier_summary* summary);

/* The same stage with every array on the device (`device` of the handle): labels in,
 * size_hist / incident (int64[V]), sub_labels (int32[V], L2) and flags (uint8[V]) out,
 * each output nullable; no host staging (the pipeline form: labels straight from
 * lpa_run(..., out_is_device = 1), results consumed on the GPU). */
int lpa_outlier_device(lpa_graph* g, const int32_t* labels, int32_t mode, int32_t sub_iter,
                       int64_t* size_hist, int64_t* incident, int32_t* sub_labels, uint8_t* flags,
                       lpa_outlier_summary* summary);

/* Partition quality of a labelling (dense ids, values in [0, V)) on the handle's
 * symmetrised multigraph, the graph labelPropagation votes on (A = 2m arcs: every
 * input edge both ways, a self-loop as two arcs at its vertex):
 *   modularity = intra_arcs / A - degree_term,  degree_term = sum_c (D_c / A)^2,
 * D_c the degree sum of community c, plus the community count (the distinct-label
 * count of Graphframes.py:85).  Exact integer sums on the device.  North-star
 * "community-count / modularity agreement" report; not a GraphFrames call.
 * On a distributed job (nranks > 1) only rank 0 keeps the edge list this needs; the
 * other ranks return LPA_EINVAL. */
typedef struct lpa_quality_summary {
  int64_t n_communities;
  int64_t intra_arcs;
  int64_t arcs;
  double degree_term;
  double modularity;
} lpa_quality_summary;
int lpa_quality(lpa_graph* g, const int32_t* labels, int32_t labels_on_device, lpa_quality_summary* out);

/* Symmetrised degree of every vertex (dense ids), host output. */
int lpa_degrees(lpa_graph* g, int32_t* deg_out);

/* lpa_graph_info has grown across header versions (it carries no size field of its
 * own; fields are only ever appended).  lpa_graph_get_info is frozen at the ABI-5
 * struct: it writes the fields up to blocked_pieces, never more, so a caller built
 * against that header is not overrun.  lpa_graph_get_info_sized(g, info, sizeof *info)
 * writes min(info_size, sizeof) bytes of this header's struct and zeroes the rest of a
 * larger caller struct: use it for the later fields.  lpa_abi_version() returns the
 * library's LPA_ABI_VERSION, so a binding can check the header it was built for.
 * ABI 7: lpa_graph_create_hostcoll, host_allgathers, the frozen unsized get_info. */
#define LPA_ABI_VERSION 7
int lpa_abi_version(void);
int lpa_graph_get_info(const lpa_graph* g, lpa_graph_info* info);
int lpa_graph_get_info_sized(const lpa_graph* g, lpa_graph_info* info, int64_t info_size);
void lpa_graph_destroy(lpa_graph* g);
const char* lpa_last_error(void);

/* ---- synthetic inputs; device outputs, caller-allocated ---- */
/* R-MAT, Graph500 A/B/C/D = .57/.19/.19/.05, m edges over 2^scale vertices,
 * duplicates and self-loops kept, optional seeded bijective id scramble. */
int lpa_gen_rmat(int32_t scale, int64_t m, uint64_t seed, int32_t scramble, int32_t* d_src,
                 int32_t* d_dst, int32_t device, void* hip_stream);
/* planted-partition SBM: V vertices in `blocks` equal blocks, p_in as a Q32 fraction. */
int lpa_gen_sbm(int32_t V, int32_t blocks, int64_t m, uint32_t p_in_q32, uint64_t seed,
                int32_t* d_src, int32_t* d_dst, int32_t device, void* hip_stream);
/* Chung-Lu power-law (config C5: "Twitter-shaped", heavy hubs): both endpoints drawn
 * with P(i) ~ (i + i0)^(-1/(gamma-1)), i0 chosen so the expected maximum degree is
 * max_deg (<= 0: i0 = 1), ranks mapped to ids by a seeded affine permutation mod V;
 * duplicates and self-loops kept.  Builds a (V+1) x 8 B weight table on the host. */
int lpa_gen_chunglu(int32_t V, int64_t m, double gamma, double max_deg, uint64_t seed,
                    int32_t* d_src, int32_t* d_dst, int32_t device, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* LPA_H_ */

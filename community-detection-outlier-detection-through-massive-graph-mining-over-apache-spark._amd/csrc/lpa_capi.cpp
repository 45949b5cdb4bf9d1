// C ABI of liblpa_hip.so (include/lpa.h).  Handle lifetime, argument checks,
// error reporting, RCCL communicator setup.
#include <stdarg.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>

#include "lpa_internal.h"

namespace lpa {

namespace {
thread_local char g_err[1024] = "";
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// carve bytes (256-B aligned) from the arena of the handle g allocates from; a block of
// max(bytes, 256 MB) is added when the current ones are exhausted
static int arena_alloc(lpa_graph* g, void** p, size_t bytes) {
  lpa_graph* o = g->arena_from;
  if (!o->arena) {
    o->arena = new (std::nothrow) Arena();
    if (!o->arena) {
      set_error("host allocation failed");
      return LPA_ENOMEM;
    }
  }
  Arena& a = *o->arena;
  bytes = (bytes + 255) & ~(size_t)255;
  while (a.cur < a.nblocks && a.off + bytes > a.blocks[a.cur].bytes) {
    ++a.cur;
    a.off = 0;
  }
  if (a.cur == a.nblocks) {
    if (a.nblocks == (int)(sizeof(a.blocks) / sizeof(a.blocks[0]))) {
      set_error("L2 sub-graph arena: too many blocks");
      return LPA_ENOMEM;
    }
    const size_t bb = bytes > ((size_t)256 << 20) ? bytes : ((size_t)256 << 20);
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, bb);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      set_error("hipMalloc(%zu bytes) for the L2 arena failed: %s", bb, hipGetErrorString(e));
      return LPA_ENOMEM;
    }
    a.blocks[a.nblocks++] = {static_cast<char*>(q), bb};
    o->device_bytes += (int64_t)bb;
    a.off = 0;
  }
  *p = a.blocks[a.cur].p + a.off;
  a.off += bytes;
  return LPA_OK;
}

void arena_reset(lpa_graph* owner) {
  if (owner->arena) {
    owner->arena->cur = 0;
    owner->arena->off = 0;
  }
}

int dev_alloc(lpa_graph* g, void** p, size_t bytes) {
  if (bytes == 0) bytes = 1;
  if (g->arena_from) {
    LPA_TRY(arena_alloc(g, p, bytes));
    g->device_bytes += (int64_t)bytes;
    return LPA_OK;
  }
  if (g->pooled) {
    LPA_TRY(tmp_alloc(p, bytes, g->stream));
    g->device_bytes += (int64_t)bytes;
    return LPA_OK;
  }
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    *p = nullptr;
    (void)hipGetLastError();
    set_error("hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
    return LPA_ENOMEM;
  }
  g->device_bytes += (int64_t)bytes;
  return LPA_OK;
}

void dev_free(lpa_graph* g, void* p) {
  if (!p || g->arena_from) return;   // arena memory goes back with the next reset
  if (g->pooled) tmp_free(p, g->stream);
  else (void)hipFree(p);
}

int scratch_alloc(lpa_graph* g, void** p, size_t bytes) {
  if (g->arena_from) return arena_alloc(g, p, bytes > 0 ? bytes : 1);
  if (g->pooled) return tmp_alloc(p, bytes > 0 ? bytes : 1, g->stream);
  hipError_t e = hipMalloc(p, bytes > 0 ? bytes : 1);
  if (e != hipSuccess) {
    *p = nullptr;
    (void)hipGetLastError();
    set_error("hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
    return LPA_ENOMEM;
  }
  return LPA_OK;
}

void scratch_free(lpa_graph* g, void* p) {
  if (!p || g->arena_from) return;
  if (g->pooled) tmp_free(p, g->stream);
  else (void)hipFree(p);
}

int gen_rmat(int32_t scale, int64_t m, uint64_t seed, int32_t do_scramble, int32_t* d_src,
             int32_t* d_dst, hipStream_t s);
int gen_sbm(int32_t V, int32_t blocks, int64_t m, uint32_t p_in_q32, uint64_t seed, int32_t* d_src,
            int32_t* d_dst, hipStream_t s);
int gen_chunglu(int32_t V, int64_t m, double gamma, double max_deg, uint64_t seed, int32_t* d_src,
                int32_t* d_dst, hipStream_t s);

void destroy(lpa_graph* g) {
  if (g) exchange_free(g);
  if (g) loopback_detach(g);
  if (g)
    for (auto& ge : g->gexec)
      if (ge) (void)hipGraphExecDestroy(ge);
  if (!g) return;
  (void)hipSetDevice(g->device);
  if (g->stream) (void)hipStreamSynchronize(g->stream);
  void* bufs[] = {g->rp,   g->col,   g->new_of, g->old_of, g->deg,   g->lab[0], g->lab[1],
                  g->segs, g->e_src,  g->e_dst, g->gsend, g->gbm, g->xpair, g->dsend, g->drecv, g->dcount, g->de_keys, g->de_t, g->de_ts, g->de_out_off, g->de_in_off, g->al,   g->cptr,  g->cpos,   g->cch, g->cowner, g->chflag, g->chlist,
                  g->counters, g->hub_best, g->hub_wcount, g->stage, g->scat, g->dev_err,
                  g->hub_hoff, g->ghist, g->gcur, g->hub_lists, g->hub_lcnt, g->hub_tickets, g->items_cb,
                  g->items_cc, g->hub_uoff, g->ucnt, g->crow, g->rdirty[0], g->rdirty[1],
                  g->udirty[0], g->udirty[1], g->fr_all, g->flist, g->ulist, g->fcnt, g->first_best, g->rstart,
                  g->blk_pieces, g->gbits, g->ugc, g->umx, g->ulist2, g->gdec, g->gword, g->al0, g->abits,
                  g->glist, g->code2, g->al2};
  for (void* p : bufs) dev_free(g, p);
  if (!g->borrowed) {   // a borrowing L2 sub-graph uses its parent's pinned words
    if (g->h_flag) (void)hipHostFree(g->h_flag);
    if (g->h_err) (void)hipHostFree(g->h_err);
  }
  if (g->arena) {
    for (int i = 0; i < g->arena->nblocks; ++i) (void)hipFree(g->arena->blocks[i].p);
    delete g->arena;
  }
  for (auto& e : g->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : g->bin_ev)
    if (e) (void)hipEventDestroy(e);
  if (!g->borrowed) {
    for (auto& st : g->aux_stream)
      if (st) (void)hipStreamDestroy(st);
    for (hipEvent_t e : {g->ev_fork, g->ev_join[0], g->ev_join[1], g->ev_fork2, g->ev_join2[0],
                         g->ev_join2[1], g->ev_join2[2]})
      if (e) (void)hipEventDestroy(e);
  }
  if (g->host_pin) (void)hipHostFree(g->host_pin);
  if (g->hc_buf) (void)hipHostFree(g->hc_buf);
  if (g->comm) (void)ncclCommDestroy(g->comm);
  if (g->own_stream) (void)hipStreamDestroy(g->own_stream);
  delete g;
}

static int check_device(int32_t device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) {
    (void)hipGetLastError();
    set_error("no HIP device available (%s)", e != hipSuccess ? hipGetErrorString(e) : "0 devices");
    return LPA_ENODEV;
  }
  if (device < 0 || device >= n) {
    set_error("device %d out of range [0, %d)", device, n);
    return LPA_ENODEV;
  }
  return LPA_OK;
}

static int check_edges(const int32_t* src, const int32_t* dst, int64_t m, int32_t V) {
  if (V < 0 || m < 0) {
    set_error("V and m must be non-negative (V=%d, m=%lld)", V, (long long)m);
    return LPA_EINVAL;
  }
  if (m > 0 && (!src || !dst)) {
    set_error("src/dst must be non-null when m > 0");
    return LPA_EINVAL;
  }
  if (m > ((int64_t)1 << 32) - 2) {
    set_error("m=%lld exceeds the supported edge count", (long long)m);
    return LPA_EINVAL;
  }
  return LPA_OK;
}

int create_common(int32_t device, hipStream_t stream, const int32_t* src, const int32_t* dst,
                  int64_t m, int32_t V, uint32_t flags, int32_t rank, int32_t nranks,
                  const uint8_t* comm_id, Loopback* loop, lpa_graph** out,
                  const lpa_graph* borrow = nullptr, const lpa_graph* l2_parent = nullptr,
                  const int32_t* l2_labels = nullptr, const uint8_t* l2_marks = nullptr,
                  lpa_allgather_fn hc_fn = nullptr, void* hc_ctx = nullptr) {
  if (!out) {
    set_error("out must be non-null");
    return LPA_EINVAL;
  }
  *out = nullptr;
  LPA_TRY(check_edges(src, dst, m, V));
  if (nranks < 1 || rank < 0 || rank >= nranks) {
    set_error("bad rank %d / nranks %d", rank, nranks);
    return LPA_EINVAL;
  }
  LPA_TRY(check_device(device));
  LPA_HIP(hipSetDevice(device));
  lpa_graph* g = new (std::nothrow) lpa_graph();
  if (!g) {
    set_error("host allocation failed");
    return LPA_ENOMEM;
  }
  g->device = device;
  if (const char* f = getenv("LPA_REBUILD_HOT")) g->rebuild_hot = atoi(f);
  if (const char* f = getenv("LPA_SERIAL")) g->serial = atoi(f);
  if (const char* f = getenv("LPA_LOCALITY")) g->locality = atoi(f);
  if (const char* f = getenv("LPA_BLOCK_DEG")) g->block_deg = atoi(f);
  if (const char* f = getenv("LPA_BLOCK_MIN_SLOTS")) g->block_min_slots = atoll(f);
  if (const char* f = getenv("LPA_GRAPHS")) g->use_graphs = atoi(f);
  if (const char* f = getenv("LPA_FRONTIER")) g->frontier = atoi(f) ? 1 : 0;
  if (const char* f = getenv("LPA_FIRST_RUNS")) g->first_runs = atoi(f) ? 1 : 0;
  if (const char* f = getenv("LPA_CODE_LBIN")) g->code_lbin_env = atoi(f);
  if (const char* f = getenv("LPA_POW2_SLICES")) g->pow2_slices = atoi(f) ? 1 : 0;
  if (const char* f = getenv("LPA_GIANT_CODES")) g->codes_env = atoi(f) ? 1 : 0;
  if (const char* f = getenv("LPA_FUSED_BINS")) g->fused_bins = atoi(f) < 0 ? 0 : atoi(f) > 2 ? 2 : atoi(f);
  if (const char* f = getenv("LPA_UNITS_PURE")) g->units_pure = atoi(f) ? 1 : 0;
  if (const char* f = getenv("LPA_KEEP_BITS")) g->keep_bits = atoi(f) ? 1 : 0;
  if (const char* f = getenv("LPA_CONV_STREAMS")) g->conv_streams = atoi(f) < 1 ? 1 : atoi(f) > 3 ? 3 : atoi(f);
  // internal builds (the outlier stage's L2 sub-graph): the locality order is a
  // gather-locality heuristic worth its two atomic passes only on a graph that runs
  // many supersteps; labels do not depend on the vertex order
  if (flags & kFlagNoLocality) g->locality = 0;
  g->pooled = (flags & kFlagPooled) && stream != nullptr;
  g->rank = rank;
  g->nranks = nranks;
  g->hc_fn = hc_fn;
  g->hc_ctx = hc_ctx;
  if (stream) {
    g->stream = stream;
  } else {
    hipError_t e = hipStreamCreateWithFlags(&g->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      set_error("hipStreamCreate: %s", hipGetErrorString(e));
      delete g;
      return LPA_EHIP;
    }
    g->stream = g->own_stream;
  }
  if (borrow) {
    // a handle used strictly in sequence with `borrow` on its stream (the outlier
    // stage's L2 sub-graph): its aux streams and fork/join events are the parent's
    // (creating and destroying three streams per call cost ~10 ms)
    for (int i = 0; i < 3; ++i) g->aux_stream[i] = borrow->aux_stream[i];
    g->ev_fork = borrow->ev_fork;
    g->ev_join[0] = borrow->ev_join[0];
    g->ev_join[1] = borrow->ev_join[1];
    g->ev_fork2 = borrow->ev_fork2;
    for (int i = 0; i < 3; ++i) g->ev_join2[i] = borrow->ev_join2[i];
    g->borrowed = true;
    g->h_flag = borrow->h_flag;   // pinned words (hipHostFree costs ~1 ms per call)
    g->h_err = borrow->h_err;
  } else {
    hipError_t e = hipSuccess;
    for (auto& st : g->aux_stream)
      if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    for (hipEvent_t* ev : {&g->ev_fork, &g->ev_join[0], &g->ev_join[1], &g->ev_fork2, &g->ev_join2[0],
                           &g->ev_join2[1], &g->ev_join2[2]})
      if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      set_error("stream/event creation: %s", hipGetErrorString(e));
      destroy(g);
      return LPA_EHIP;
    }
  }
  if (loop) {
    int rc = loopback_attach(g, loop);
    if (rc != LPA_OK) {
      destroy(g);
      return rc;
    }
  } else if (comm_id) {
    ncclUniqueId id;
    memcpy(&id, comm_id, sizeof(id));
    ncclResult_t r = ncclCommInitRank(&g->comm, nranks, id, rank);
    if (r != ncclSuccess) {
      set_error("ncclCommInitRank(rank %d of %d): %s", rank, nranks, ncclGetErrorString(r));
      g->comm = nullptr;
      destroy(g);
      return LPA_ERCCL;
    }
  }
  if (l2_parent) {   // every array of the sub-graph from the parent's arena (reset here)
    g->arena_from = const_cast<lpa_graph*>(l2_parent);
    arena_reset(g->arena_from);
  }
  int rc = l2_parent ? build_graph_l2(g, l2_parent, l2_labels, l2_marks) : build_graph(g, src, dst, m, V, flags);
  if (rc == LPA_OK) rc = exchange_alloc(g);
  if (rc != LPA_OK) {
    destroy(g);
    return rc;
  }
  *out = g;
  return LPA_OK;
}

// the outlier stage's L2 sub-graph of `parent` under the community labels L (device,
// dense ids): pooled, on the parent's stream, borrowing its aux streams
int create_l2(const lpa_graph* parent, const int32_t* L, const uint8_t* marks, lpa_graph** out) {
  return create_common(parent->device, parent->stream, nullptr, nullptr, 0, (int32_t)parent->V,
                       kFlagNoLocality | kFlagPooled, 0, 1, nullptr, nullptr, out, parent, parent, L, marks);
}

}  // namespace lpa

using namespace lpa;

extern "C" {

const char* lpa_last_error(void) { return g_err; }

int lpa_graph_create(const int32_t* src, const int32_t* dst, int64_t m, int32_t V, int32_t device,
                     uint32_t flags, lpa_graph** out) {
  return create_common(device, nullptr, src, dst, m, V, flags, 0, 1, nullptr, nullptr, out);
}

int lpa_comm_unique_id(uint8_t id_out[128]) {
  if (!id_out) {
    set_error("id_out must be non-null");
    return LPA_EINVAL;
  }
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    set_error("ncclGetUniqueId: %s", ncclGetErrorString(r));
    return LPA_ERCCL;
  }
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  memcpy(id_out, &id, 128);
  return LPA_OK;
}

int lpa_graph_create_dist(const int32_t* src, const int32_t* dst, int64_t m, int32_t V,
                          int32_t device, uint32_t flags, int32_t rank, int32_t nranks,
                          const uint8_t comm_id[128], lpa_graph** out) {
  return create_common(device, nullptr, src, dst, m, V, flags, rank, nranks, comm_id, nullptr, out);
}

int lpa_graph_create_loopback(const int32_t* src, const int32_t* dst, int64_t m, int32_t V,
                              int32_t device, uint32_t flags, int32_t rank, lpa_loopback* group,
                              lpa_graph** out) {
  if (!group) {
    set_error("lpa_graph_create_loopback: null group");
    return LPA_EINVAL;
  }
  Loopback* lb = reinterpret_cast<Loopback*>(group);
  return create_common(device, nullptr, src, dst, m, V, flags, rank, loopback_ranks(lb), nullptr, lb,
                       out);
}

int lpa_graph_create_hostcoll(const int32_t* src, const int32_t* dst, int64_t m, int32_t V, int32_t device,
                              uint32_t flags, int32_t rank, int32_t nranks, lpa_allgather_fn allgather, void* ctx,
                              lpa_graph** out) {
  if (!allgather) {
    set_error("lpa_graph_create_hostcoll: null allgather function");
    return LPA_EINVAL;
  }
  return create_common(device, nullptr, src, dst, m, V, flags, rank, nranks, nullptr, nullptr, out, nullptr,
                       nullptr, nullptr, nullptr, allgather, ctx);
}

int lpa_exchange_get(lpa_graph* g, int32_t* slice_out) {
  if (!g || !slice_out) {
    set_error("null handle or output");
    return LPA_EINVAL;
  }
  LPA_HIP(hipSetDevice(g->device));
  LPA_HIP(hipMemcpyAsync(slice_out, g->lab[g->cur] + g->own_begin, sizeof(int32_t) * g->slice,
                         hipMemcpyDeviceToHost, g->stream));
  LPA_HIP(hipStreamSynchronize(g->stream));
  return LPA_OK;
}

int lpa_exchange_put(lpa_graph* g, const int32_t* full_in) {
  if (!g || !full_in) {
    set_error("null handle or input");
    return LPA_EINVAL;
  }
  LPA_HIP(hipSetDevice(g->device));
  LPA_HIP(hipMemcpyAsync(g->lab[g->cur], full_in, sizeof(int32_t) * g->vpad, hipMemcpyHostToDevice,
                         g->stream));
  g->prev_delta_ok = false;
  LPA_TRY(refresh_after_put(g));
  g->al_pending = false;
  LPA_TRY(frontier_all(g, g->par));
  LPA_HIP(hipStreamSynchronize(g->stream));
  return LPA_OK;
}

int lpa_exchange_get_delta(lpa_graph* g, uint64_t* entries_out, int64_t* count_out) {
  if (!g || !entries_out || !count_out || g->nranks <= 1) {
    set_error("lpa_exchange_get_delta: null argument or single-rank handle");
    return LPA_EINVAL;
  }
  LPA_HIP(hipSetDevice(g->device));
  // after lpa_step the current vector holds this rank's new owned labels, the other
  // one the labels they replace
  LPA_TRY(exchange_compact(g, g->lab[g->cur ^ 1], g->lab[g->cur]));
  unsigned long long n = 0;
  LPA_HIP(hipMemcpyAsync(&n, g->dcount, sizeof(n), hipMemcpyDeviceToHost, g->stream));
  LPA_HIP(hipStreamSynchronize(g->stream));
  if (n > 0)
    LPA_HIP(hipMemcpyAsync(entries_out, g->dsend, sizeof(uint64_t) * n, hipMemcpyDeviceToHost,
                           g->stream));
  LPA_HIP(hipStreamSynchronize(g->stream));
  *count_out = (int64_t)n;
  return LPA_OK;
}

int lpa_exchange_put_delta(lpa_graph* g, const uint64_t* entries, const int64_t* counts, int64_t cap) {
  if (!g || !counts || (cap > 0 && !entries) || g->nranks <= 1 || cap < 0) {
    set_error("lpa_exchange_put_delta: null argument or single-rank handle");
    return LPA_EINVAL;
  }
  if (cap > g->dcap) {
    set_error("lpa_exchange_put_delta: %lld entries per rank exceed the delta capacity %lld "
              "(use lpa_exchange_put)", (long long)cap, (long long)g->dcap);
    return LPA_EINVAL;
  }
  for (int r = 0; r < g->nranks; ++r)
    if (counts[r] < 0 || counts[r] > cap) {
      set_error("lpa_exchange_put_delta: count of rank %d out of [0, cap]", r);
      return LPA_EINVAL;
    }
  LPA_HIP(hipSetDevice(g->device));
  hipStream_t s = g->stream;
  // the receive buffer lays entries out as [nranks][cap] like the RCCL allgather
  if (cap > 0)
    LPA_HIP(hipMemcpyAsync(exchange_recv_buf(g), entries, sizeof(uint64_t) * cap * g->nranks,
                           hipMemcpyHostToDevice, s));
  LPA_HIP(hipMemcpyAsync(exchange_recv_counts(g), counts, sizeof(int64_t) * g->nranks,
                         hipMemcpyHostToDevice, s));
  // this refresh completes the superstep that just ran (lpa_step already flipped the
  // parity): its counters (zeroed here -- the caller-driven path runs no scatter of
  // its own), its arc mode, and the next superstep's flags / mode
  const int pp = g->par ^ 1;
  LPA_TRY(ensure_al(g));   // the scatter below updates al in place
  LPA_HIP(hipMemsetAsync(g->counters + 4 * pp, 0, sizeof(unsigned long long) * 2, s));
  const int32_t* Lc = g->lab[g->cur ^ 1];
  int32_t* Ln = g->lab[g->cur];
  LPA_TRY(exchange_finish_delta(g, const_cast<int32_t*>(Lc), Ln, cap, pp, exchange_recv_counts(g), 1));
  LPA_TRY(launch_refresh_ext(g, Lc, Ln, true, pp));
  LPA_HIP(hipStreamSynchronize(s));
  return LPA_OK;
}

int lpa_set_serial(lpa_graph* g, int32_t serial) {
  if (!g) {
    set_error("null handle");
    return LPA_EINVAL;
  }
  g->serial = serial ? 1 : 0;
  return LPA_OK;
}

int lpa_set_posted(lpa_graph* g, int64_t cap) {
  if (!g) {
    set_error("null handle");
    return LPA_EINVAL;
  }
  g->post_fixed = cap < 0 ? -1 : cap;
  return LPA_OK;
}

int lpa_set_frontier(lpa_graph* g, int32_t on) {
  if (!g) {
    set_error("null handle");
    return LPA_EINVAL;
  }
  on = on ? 1 : 0;
  if (on != g->frontier) {
    LPA_HIP(hipSetDevice(g->device));
    LPA_HIP(hipStreamSynchronize(g->stream));
    // the flag is baked into the captured superstep graphs
    for (auto& ge : g->gexec)
      if (ge) {
        (void)hipGraphExecDestroy(ge);
        ge = nullptr;
      }
    g->frontier = on;
    // the next superstep tallies every row either way (flags may be stale)
    LPA_TRY(frontier_all(g, g->par));
    LPA_HIP(hipStreamSynchronize(g->stream));
  }
  return LPA_OK;
}

int lpa_set_stream(lpa_graph* g, void* hip_stream) {
  if (!g) {
    set_error("null handle");
    return LPA_EINVAL;
  }
  LPA_HIP(hipSetDevice(g->device));
  LPA_HIP(hipStreamSynchronize(g->stream));
  g->stream = hip_stream ? (hipStream_t)hip_stream : g->own_stream;
  if (!g->stream) {
    LPA_HIP(hipStreamCreateWithFlags(&g->own_stream, hipStreamNonBlocking));
    g->stream = g->own_stream;
  }
  return LPA_OK;
}

int lpa_reset(lpa_graph* g) {
  if (!g) {
    set_error("null handle");
    return LPA_EINVAL;
  }
  LPA_HIP(hipSetDevice(g->device));
  LPA_TRY(init_labels(g));
  LPA_HIP(hipStreamSynchronize(g->stream));
  return LPA_OK;
}

int lpa_step(lpa_graph* g, int32_t n_supersteps, lpa_stats* stats) {
  if (!g) {
    set_error("null handle");
    return LPA_EINVAL;
  }
  if (n_supersteps < 0) {
    set_error("n_supersteps must be >= 0, got %d", n_supersteps);
    return LPA_EINVAL;
  }
  LPA_HIP(hipSetDevice(g->device));
  return run_supersteps(g, n_supersteps, stats);
}

int lpa_get_labels(lpa_graph* g, int32_t* labels_out, int32_t out_is_device) {
  if (!g || (!labels_out && g->V > 0)) {
    set_error("null handle or output");
    return LPA_EINVAL;
  }
  LPA_HIP(hipSetDevice(g->device));
  if (g->V == 0) return LPA_OK;
  if (out_is_device) {
    LPA_TRY(gather_labels(g, labels_out));
  } else {
    int32_t* tmp = nullptr;
    LPA_HIP(hipMalloc((void**)&tmp, sizeof(int32_t) * g->V));
    int rc = gather_labels(g, tmp);
    if (rc == LPA_OK)
      LPA_HIP(hipMemcpyAsync(labels_out, tmp, sizeof(int32_t) * g->V, hipMemcpyDeviceToHost, g->stream));
    LPA_HIP(hipFree(tmp));
    if (rc != LPA_OK) return rc;
  }
  LPA_HIP(hipStreamSynchronize(g->stream));
  return LPA_OK;
}

int lpa_run(lpa_graph* g, int32_t max_iter, int32_t* labels_out, int32_t out_is_device,
            lpa_stats* stats) {
  if (!g) {
    set_error("null handle");
    return LPA_EINVAL;
  }
  if (max_iter <= 0) {
    set_error("requirement failed: Maximum of steps must be greater than 0, but got %d", max_iter);
    return LPA_EINVAL;
  }
  LPA_TRY(lpa_reset(g));
  LPA_TRY(lpa_step(g, max_iter, stats));
  if (labels_out) LPA_TRY(lpa_get_labels(g, labels_out, out_is_device));
  return LPA_OK;
}

int lpa_outlier(lpa_graph* g, const int32_t* labels, int32_t labels_on_device, int32_t mode,
                int32_t sub_iter, int64_t* size_hist, int64_t* incident, int32_t* sub_labels,
                uint8_t* flags, lpa_outlier_summary* summary) {
  if (!g || (!labels && g->V > 0)) {
    set_error("null handle or labels");
    return LPA_EINVAL;
  }
  if (g->nranks > 1) {
    set_error("lpa_outlier runs on a single-GPU handle");
    return LPA_EINVAL;
  }
  LPA_HIP(hipSetDevice(g->device));
  return outlier(g, labels, labels_on_device, mode, sub_iter, size_hist, incident, sub_labels, flags,
                 summary, 0);
}

int lpa_outlier_device(lpa_graph* g, const int32_t* labels, int32_t mode, int32_t sub_iter, int64_t* size_hist,
                       int64_t* incident, int32_t* sub_labels, uint8_t* flags, lpa_outlier_summary* summary) {
  if (!g || (!labels && g->V > 0)) {
    set_error("null handle or labels");
    return LPA_EINVAL;
  }
  if (g->nranks > 1) {
    set_error("lpa_outlier runs on a single-GPU handle");
    return LPA_EINVAL;
  }
  LPA_HIP(hipSetDevice(g->device));
  return outlier(g, labels, 1, mode, sub_iter, size_hist, incident, sub_labels, flags, summary, 1);
}

int lpa_quality(lpa_graph* g, const int32_t* labels, int32_t labels_on_device, lpa_quality_summary* out) {
  if (!g || !out || (!labels && g->V > 0)) {
    set_error("null handle, labels or output");
    return LPA_EINVAL;
  }
  if (g->m > 0 && !g->e_src) {
    set_error("lpa_quality of a distributed job runs on rank 0 (the rank that keeps the edge list)");
    return LPA_EINVAL;
  }
  LPA_HIP(hipSetDevice(g->device));
  return quality(g, labels, labels_on_device, out);
}

int lpa_degrees(lpa_graph* g, int32_t* deg_out) {
  if (!g || (!deg_out && g->V > 0)) {
    set_error("null handle or output");
    return LPA_EINVAL;
  }
  LPA_HIP(hipSetDevice(g->device));
  if (g->V > 0)
    LPA_HIP(hipMemcpyAsync(deg_out, g->deg, sizeof(int32_t) * g->V, hipMemcpyDeviceToHost, g->stream));
  LPA_HIP(hipStreamSynchronize(g->stream));
  return LPA_OK;
}

}  // extern "C"

namespace {
// every field of this header's lpa_graph_info
int fill_info(const lpa_graph* g, lpa_graph_info* info) {
  memset(info, 0, sizeof(*info));
  info->V = g->V;
  info->m = g->m;
  info->arcs = g->arcs;
  info->slice = g->slice;
  info->own_begin = g->own_begin;
  info->rank = g->rank;
  info->nranks = g->nranks;
  info->device = g->device;
  info->max_degree = g->max_degree;
  for (int b = 0; b < LPA_NBINS; ++b) {
    info->bin_vertices[b] = g->bin_begin[b + 1] - g->bin_begin[b];
    info->bin_arcs[b] = g->bin_arcs[b];
  }
  info->hub_vertices = g->n_hub;
  info->segments = g->n_segs;
  info->device_bytes = g->device_bytes;
  info->exchanges_full = g->n_exch_full;
  info->exchanges_delta = g->n_exch_delta;
  info->exchanges_giant = g->n_exch_giant;
  info->blocked_rows = g->blk_pieces ? g->blk_rows : 0;
  info->blocked_pieces = g->blk_pieces ? g->blk_off[g->blk_classes] : 0;
  info->graph_replays = g->n_graph_replays;
  info->exchanges_posted = g->n_exch_posted;
  info->exchanges_post_missed = g->n_exch_post_missed;
  info->gather_mode = g->gather ? 1 : 0;
  info->host_allgathers = g->n_host_allgathers;
  if (g->code_ok && g->gword) {
    LPA_HIP(hipSetDevice(g->device));
    int32_t w = 0;
    LPA_HIP(hipMemcpyAsync(&w, g->gword + 5, sizeof(int32_t), hipMemcpyDeviceToHost, g->stream));
    LPA_HIP(hipStreamSynchronize(g->stream));
    info->code_refresh = w;
  }
  return LPA_OK;
}
}  // namespace

extern "C" {

// the unsized form is frozen at the ABI-5 struct (the fields up to blocked_pieces): a
// caller compiled against that header passes a struct of that size
int lpa_graph_get_info(const lpa_graph* g, lpa_graph_info* info) {
  if (!g || !info) {
    set_error("null handle or info");
    return LPA_EINVAL;
  }
  lpa_graph_info full;
  LPA_TRY(fill_info(g, &full));
  memcpy(info, &full, offsetof(lpa_graph_info, code_refresh));
  return LPA_OK;
}

int lpa_abi_version(void) { return LPA_ABI_VERSION; }

int lpa_graph_get_info_sized(const lpa_graph* g, lpa_graph_info* info, int64_t info_size) {
  if (!g || !info || info_size < 0) {
    set_error("null handle, null info or negative size");
    return LPA_EINVAL;
  }
  lpa_graph_info full;
  LPA_TRY(fill_info(g, &full));
  // a caller's struct from a later header: the fields this library does not know read 0
  if (info_size > (int64_t)sizeof(full)) memset(reinterpret_cast<char*>(info) + sizeof(full), 0,
                                                (size_t)info_size - sizeof(full));
  memcpy(info, &full, (size_t)(info_size < (int64_t)sizeof(full) ? info_size : (int64_t)sizeof(full)));
  return LPA_OK;
}

void lpa_graph_destroy(lpa_graph* g) {
  if (!g) return;
  const int dev = g->device;
  destroy(g);
  tmp_trim(dev);  // the stream-ordered temporaries' cached memory goes back to the device
}

int lpa_gen_rmat(int32_t scale, int64_t m, uint64_t seed, int32_t scramble, int32_t* d_src,
                 int32_t* d_dst, int32_t device, void* hip_stream) {
  LPA_TRY(check_device(device));
  LPA_HIP(hipSetDevice(device));
  if (m > 0 && (!d_src || !d_dst)) {
    set_error("d_src/d_dst must be non-null");
    return LPA_EINVAL;
  }
  hipStream_t s = (hipStream_t)hip_stream;
  LPA_TRY(gen_rmat(scale, m, seed, scramble, d_src, d_dst, s));
  LPA_HIP(hipStreamSynchronize(s));
  return LPA_OK;
}

int lpa_gen_sbm(int32_t V, int32_t blocks, int64_t m, uint32_t p_in_q32, uint64_t seed,
                int32_t* d_src, int32_t* d_dst, int32_t device, void* hip_stream) {
  LPA_TRY(check_device(device));
  LPA_HIP(hipSetDevice(device));
  if (m > 0 && (!d_src || !d_dst)) {
    set_error("d_src/d_dst must be non-null");
    return LPA_EINVAL;
  }
  hipStream_t s = (hipStream_t)hip_stream;
  LPA_TRY(gen_sbm(V, blocks, m, p_in_q32, seed, d_src, d_dst, s));
  LPA_HIP(hipStreamSynchronize(s));
  return LPA_OK;
}

int lpa_gen_chunglu(int32_t V, int64_t m, double gamma, double max_deg, uint64_t seed,
                    int32_t* d_src, int32_t* d_dst, int32_t device, void* hip_stream) {
  LPA_TRY(check_device(device));
  LPA_HIP(hipSetDevice(device));
  if (m > 0 && (!d_src || !d_dst)) {
    set_error("d_src/d_dst must be non-null");
    return LPA_EINVAL;
  }
  hipStream_t s = (hipStream_t)hip_stream;
  LPA_TRY(gen_chunglu(V, m, gamma, max_deg, seed, d_src, d_dst, s));
  LPA_HIP(hipStreamSynchronize(s));
  return LPA_OK;
}

}  // extern "C"

// Collective backend of the multi-GPU label exchange (replaces the
// Spark shuffle behind aggregateMessages).
//
//   RCCL      ncclAllGather on the handle's communicator: one process per GPU,
//             xGMI between ranks (lpa_graph_create_dist with a comm id).
//   loopback  an in-process group of P handles on ONE device, each driven by its
//             own host thread exactly as P processes would drive theirs
//             (lpa_graph_create_loopback).  The allgather is stream-ordered D2D
//             copies: every rank publishes its send buffer and a "ready" event,
//             meets the others at a host barrier, pulls every slice into its own
//             receive buffer on its own stream, records a "done" event, and after a
//             second barrier makes its stream wait for every other rank's copies
//             (so its next write to the send buffer cannot race a peer's read).
//             This runs the library's exchange control flow -- dense/delta switch,
//             host count read, in-place allgather offsets, delta chain -- on a
//             one-GPU box, where RCCL refuses two ranks on one device.
//   host      (round 6) the caller's host function (lpa_graph_create_hostcoll): the
//             send bytes are staged to pinned host memory, the function gathers every
//             rank's bytes in rank order (torch.distributed gloo, MPI, a Spark barrier
//             stage ...), the result is copied back -- the library's exchange schedule,
//             every form included, across real process boundaries without RCCL.
#include <condition_variable>
#include <chrono>
#include <mutex>
#include <new>
#include <vector>

#include "lpa_internal.h"

namespace lpa {

struct Loopback {
  int P = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<lpa_graph*> rank_g;   // attached handles
  std::vector<const void*> send;    // published send buffers (current collective)
  std::vector<size_t> bytes;        // published bytes per rank (must agree)
  int timeout_s = 300;
  int attached = 0;                 // handles attached (rank_g non-null)
  bool destroy_pending = false;     // lpa_loopback_destroy while handles were attached:
                                    // the last detach frees the group

  // returns false on abort / timeout (the group is then poisoned: every later
  // collective fails fast instead of hanging the other ranks' threads)
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return false;
    const uint64_t my = gen;
    if (++arrived == P) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    const bool ok = cv.wait_for(lk, std::chrono::seconds(timeout_s),
                                [&] { return gen != my || aborted; });
    if (!ok || aborted) {
      aborted = true;
      cv.notify_all();
      return false;
    }
    return true;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
};

int loopback_ranks(const Loopback* lb) { return lb ? lb->P : 0; }

int loopback_attach(lpa_graph* g, Loopback* lb) {
  if (!lb || g->rank >= lb->P || g->nranks != lb->P) {
    set_error("loopback group of %d ranks cannot take rank %d of %d", lb ? lb->P : 0, g->rank,
              g->nranks);
    return LPA_EINVAL;
  }
  std::lock_guard<std::mutex> lk(lb->mu);
  if (lb->rank_g[g->rank]) {
    set_error("loopback rank %d is already attached", g->rank);
    return LPA_EINVAL;
  }
  if (lb->destroy_pending) {
    set_error("loopback group is being destroyed");
    return LPA_EINVAL;
  }
  // events last: an error return above leaves nothing to release (g->loop stays null,
  // so loopback_detach would not destroy them)
  for (auto& e : g->loop_ev) {
    const hipError_t er = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (er != hipSuccess) {
      for (auto& f : g->loop_ev)
        if (f) {
          (void)hipEventDestroy(f);
          f = nullptr;
        }
      set_error("hipEventCreateWithFlags failed: %s", hipGetErrorString(er));
      return LPA_EHIP;
    }
  }
  lb->rank_g[g->rank] = g;
  ++lb->attached;
  g->loop = lb;
  return LPA_OK;
}

void loopback_detach(lpa_graph* g) {
  Loopback* lb = g->loop;
  if (!lb) return;
  bool last = false;
  {
    std::lock_guard<std::mutex> lk(lb->mu);
    if (lb->rank_g[g->rank] == g) {
      lb->rank_g[g->rank] = nullptr;
      --lb->attached;
    }
    last = lb->destroy_pending && lb->attached == 0;
  }
  for (auto& e : g->loop_ev)
    if (e) (void)hipEventDestroy(e);
  g->loop = nullptr;
  if (last) delete lb;  // the group was destroyed while this handle was attached
}

namespace {

int loop_allgather(lpa_graph* g, const void* send, void* recv, size_t bytes, hipStream_t s) {
  Loopback* lb = g->loop;
  const int r = g->rank, P = lb->P;
  LPA_HIP(hipEventRecord(g->loop_ev[0], s));  // this rank's send data is ready
  {
    std::lock_guard<std::mutex> lk(lb->mu);
    lb->send[r] = send;
    lb->bytes[r] = bytes;
  }
  if (!lb->barrier()) {
    set_error("loopback allgather: a peer rank did not arrive (aborted or timed out)");
    return LPA_ERCCL;
  }
  for (int q = 0; q < P; ++q) {
    if (lb->bytes[q] != bytes || !lb->rank_g[q]) {
      lb->abort();
      set_error("loopback allgather: rank %d sent %zu bytes, rank %d expects %zu", q, lb->bytes[q], r,
                bytes);
      return LPA_ERCCL;
    }
  }
  char* dst = static_cast<char*>(recv);
  for (int q = 0; q < P; ++q) {
    char* to = dst + (size_t)q * bytes;
    if (bytes == 0 || to == lb->send[q]) continue;  // in place (own slice)
    if (q != r) LPA_HIP(hipStreamWaitEvent(s, lb->rank_g[q]->loop_ev[0], 0));
    LPA_HIP(hipMemcpyAsync(to, lb->send[q], bytes, hipMemcpyDeviceToDevice, s));
  }
  LPA_HIP(hipEventRecord(g->loop_ev[1], s));  // this rank's reads of the peers are queued
  if (!lb->barrier()) {
    set_error("loopback allgather: a peer rank did not arrive (aborted or timed out)");
    return LPA_ERCCL;
  }
  for (int q = 0; q < P; ++q)
    if (q != r) LPA_HIP(hipStreamWaitEvent(s, lb->rank_g[q]->loop_ev[1], 0));
  // third meeting: every rank has queued its waits on the others' events, so no rank
  // runs ahead into a stream capture (the converged supersteps' captured tally) while a
  // peer still makes its stream wait on an event of the capturing stream -- the runtime
  // refuses that ("dependency created on uncaptured work")
  if (!lb->barrier()) {
    set_error("loopback allgather: a peer rank did not arrive (aborted or timed out)");
    return LPA_ERCCL;
  }
  return LPA_OK;
}

// The host collective: stream-ordered up to the staging copies, synchronous around the
// caller's function (it runs on this host thread; the staging buffer is reused by the
// next allgather, so the copy back completes before returning)
int host_allgather(lpa_graph* g, const void* send, void* recv, size_t bytes, hipStream_t s) {
  const int P = g->nranks;
  const size_t need = bytes * (size_t)(P + 1) > 0 ? bytes * (size_t)(P + 1) : 1;
  if (g->hc_bytes < need) {
    if (g->hc_buf) LPA_HIP(hipHostFree(g->hc_buf));
    g->hc_buf = nullptr;
    g->hc_bytes = 0;
    LPA_HIP(hipHostMalloc(&g->hc_buf, need, hipHostMallocDefault));
    g->hc_bytes = need;
  }
  char* hs = static_cast<char*>(g->hc_buf);
  char* hr = hs + bytes;
  if (bytes > 0) LPA_HIP(hipMemcpyAsync(hs, send, bytes, hipMemcpyDeviceToHost, s));
  LPA_HIP(hipStreamSynchronize(s));
  const int rc = g->hc_fn(hs, hr, (int64_t)bytes, g->hc_ctx);
  if (rc != 0) {
    set_error("host allgather function failed (returned %d) on rank %d, %zu bytes per rank", rc, g->rank, bytes);
    return LPA_ERCCL;
  }
  ++g->n_host_allgathers;
  if (bytes > 0) LPA_HIP(hipMemcpyAsync(recv, hr, bytes * (size_t)P, hipMemcpyHostToDevice, s));
  LPA_HIP(hipStreamSynchronize(s));
  return LPA_OK;
}

}  // namespace

int coll_allgather(lpa_graph* g, const void* send, void* recv, size_t count, int elem, hipStream_t s) {
  if (g->hc_fn) return host_allgather(g, send, recv, count * (size_t)elem, s);
  if (g->loop) {
    int rc = loop_allgather(g, send, recv, count * (size_t)elem, s);
    if (rc != LPA_OK && g->loop) g->loop->abort();
    return rc;
  }
  const ncclDataType_t dt = elem == 8 ? ncclUint64 : elem == 4 ? ncclInt32 : ncclUint8;
  if (elem != 8 && elem != 4) count *= (size_t)elem;
  ncclResult_t r = ncclAllGather(send, recv, count, dt, g->comm, s);
  if (r != ncclSuccess) {
    set_error("ncclAllGather (%zu x %d B): %s", count, elem, ncclGetErrorString(r));
    return LPA_ERCCL;
  }
  return LPA_OK;
}

}  // namespace lpa

using namespace lpa;

extern "C" {

int lpa_loopback_create(int32_t nranks, lpa_loopback** out) {
  if (!out || nranks < 1) {
    set_error("lpa_loopback_create: nranks must be >= 1 and out non-null");
    return LPA_EINVAL;
  }
  Loopback* lb = new (std::nothrow) Loopback();
  if (!lb) {
    set_error("host allocation failed");
    return LPA_ENOMEM;
  }
  lb->P = nranks;
  lb->rank_g.assign(nranks, nullptr);
  lb->send.assign(nranks, nullptr);
  lb->bytes.assign(nranks, 0);
  *out = reinterpret_cast<lpa_loopback*>(lb);
  return LPA_OK;
}

void lpa_loopback_abort(lpa_loopback* group) {
  if (group) reinterpret_cast<Loopback*>(group)->abort();
}

// A group destroyed while handles are still attached is poisoned (their collectives
// fail fast) and freed by the last handle's detach (lpa_graph_destroy), so a handle
// never locks a freed group.
void lpa_loopback_destroy(lpa_loopback* group) {
  Loopback* lb = reinterpret_cast<Loopback*>(group);
  if (!lb) return;
  {
    std::lock_guard<std::mutex> lk(lb->mu);
    if (lb->attached > 0) {
      lb->destroy_pending = true;
      lb->aborted = true;
      lb->cv.notify_all();
      return;
    }
  }
  delete lb;
}

}  // extern "C"

// kp_multi.cpp — kp_create_multi: one context over several GPUs of a node,
// for a single manager process (the reference runs ONE manager process with
// one reconciler, cmd/manager/main.go:157-200, :181-187).
//
// Design: the context owns one single-GPU shard context per GPU
// (rank r of n: the r-th contiguous block of ranked units) and one persistent
// worker thread per shard. Every entry point of include/kplace.h forwards to
// the shards on their workers and waits for all of them; the shards run the
// same device-driven solve as the one-process-per-GPU form, exchanging their
// candidates once per round:
//   - distinct GPU ids: RCCL communicators from ncclCommInitAll, over xGMI;
//   - a repeated id (several shards on one GPU: testing on a 1-GPU box): the
//     host-staged exchange through an in-process all-gather below.
// Outputs are read from shard 0: every shard commits the identical placement
// (integer work, deterministic order).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>

#include "kp_internal.hpp"

namespace kp {

// In-process all-gather: rank r copies its block into slot r of a shared
// buffer; a generation barrier releases the ranks once every slot is filled,
// a second one holds the buffer until every rank has copied it out. A failed
// shard poisons it so that the others return instead of waiting forever.
struct InProc {
  std::mutex m;
  std::condition_variable cv;
  int n = 0, arrived = 0;
  uint64_t gen = 0;
  bool poisoned = false;
  std::vector<uint8_t> buf;

  bool barrier(std::unique_lock<std::mutex> &lk) {
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || poisoned; });
    }
    return !poisoned;
  }
  void poison() {
    std::lock_guard<std::mutex> g(m);
    poisoned = true;
    cv.notify_all();
  }
  void reset() {
    std::lock_guard<std::mutex> g(m);
    poisoned = false;
    arrived = 0;
  }
};

struct RankRef {
  InProc *ip;
  int rank;
};

static int inproc_allgather(void *user, const void *send, size_t bytes, void *recv) {
  RankRef *rr = static_cast<RankRef *>(user);
  InProc &ip = *rr->ip;
  std::unique_lock<std::mutex> lk(ip.m);
  if (ip.poisoned) return 1;
  // every rank passes the same size (the exchange block is sized by the
  // global slot bound); nobody reads the buffer between two calls
  if (ip.arrived == 0 && ip.buf.size() < bytes * ip.n) ip.buf.resize(bytes * ip.n);
  std::memcpy(ip.buf.data() + bytes * rr->rank, send, bytes);
  if (!ip.barrier(lk)) return 1;
  std::memcpy(recv, ip.buf.data(), bytes * ip.n);
  return ip.barrier(lk) ? 0 : 1;
}

struct Worker {
  std::thread th;
  std::mutex m;
  std::condition_variable cv;
  std::function<int()> job;
  bool has = false, done = false, stop = false;
  int rc = 0;
};

struct Multi {
  std::vector<kp_ctx *> shards;
  std::vector<std::unique_ptr<Worker>> workers;
  std::unique_ptr<InProc> inproc;
  std::vector<RankRef> refs;
  bool rccl = false;
  bool broken = false;  // an RCCL shard failed mid-exchange: communicators aborted
  // set by the first shard whose call fails (its index in first_fail): the
  // other shards' exchange waits poll it and return instead of hanging
  std::atomic<int> failed{0};
  std::atomic<int> first_fail{-1};
};

static void worker_loop(Worker *w, int device) {
  (void)hipSetDevice(device);
  while (true) {
    std::function<int()> job;
    {
      std::unique_lock<std::mutex> lk(w->m);
      w->cv.wait(lk, [&] { return w->has || w->stop; });
      if (w->stop) return;
      job = std::move(w->job);
      w->has = false;
    }
    const int rc = job();
    std::lock_guard<std::mutex> lk(w->m);
    w->rc = rc;
    w->done = true;
    w->cv.notify_all();
  }
}

int multi_run(kp_ctx *c, const std::function<int(kp_ctx *, int)> &fn, bool all) {
  Multi &M = *c->multi;
  std::lock_guard<std::mutex> g(c->mu);
  c->last_error.clear();
  if (M.broken) {
    c->last_error = "kp_create_multi context: an earlier RCCL failure aborted its communicators";
    return KP_ERCCL;
  }
  if (M.inproc) M.inproc->reset();
  M.failed.store(0);
  M.first_fail.store(-1);
  const int n = all ? (int)M.shards.size() : 1;
  for (int i = 0; i < n; ++i) {
    Worker &w = *M.workers[i];
    kp_ctx *sh = M.shards[i];
    std::lock_guard<std::mutex> lk(w.m);
    w.job = [&fn, sh, i, &M]() {
      const int rc = fn(sh, i);
      if (rc != KP_OK) {  // release the others at once (not after every shard returned)
        int none = -1;
        M.first_fail.compare_exchange_strong(none, i);
        M.failed.store(1, std::memory_order_release);
        if (M.inproc) M.inproc->poison();
      }
      return rc;
    };
    w.done = false;
    w.has = true;
    w.cv.notify_all();
  }
  std::vector<int> rcs(n, KP_OK);
  for (int i = 0; i < n; ++i) {
    Worker &w = *M.workers[i];
    std::unique_lock<std::mutex> lk(w.m);
    w.cv.wait(lk, [&] { return w.done; });
    rcs[i] = w.rc;
  }
  // report the root cause: the shard that failed first (its peers then fail
  // with KP_ERCCL "a peer shard failed")
  const int f = M.first_fail.load();
  if (f < 0) return KP_OK;
  const int rc = rcs[f];
  {
    std::lock_guard<std::mutex> sg(M.shards[f]->mu);
    c->last_error = "shard " + std::to_string(f) + ": " + M.shards[f]->last_error;
  }
  bool stuck = false;  // some shard has a collective in flight that may never complete
  for (int i = 0; i < n; ++i) stuck = stuck || M.shards[i]->in_collective;
  if (M.rccl && all && n > 1 && stuck) {
    // every worker has returned (no host thread is inside RCCL): abort the
    // communicators so that device-side collectives waiting for the failed
    // shard terminate; the context then reports KP_ERCCL for every call
    for (kp_ctx *sh : M.shards)
      if (sh->nccl_comm) (void)ncclCommAbort(static_cast<ncclComm_t>(sh->nccl_comm));
    for (kp_ctx *sh : M.shards) sh->nccl_comm = nullptr;
    M.broken = true;
  }
  return rc;
}

void multi_destroy(kp_ctx *c) {
  Multi *M = c->multi;
  for (auto &w : M->workers) {
    {
      std::lock_guard<std::mutex> lk(w->m);
      w->stop = true;
      w->cv.notify_all();
    }
    if (w->th.joinable()) w->th.join();
  }
  for (kp_ctx *sh : M->shards) kp_destroy(sh);
  delete M;
  delete c;
}

int multi_create(kp_ctx **out, const int32_t *ids, int32_t n, int64_t max_pairs) {
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return KP_ENODEV;
  for (int i = 0; i < n; ++i)
    if (ids[i] < 0 || ids[i] >= ndev) return KP_ENODEV;
  std::vector<int> devs(ids, ids + n);
  std::vector<int> sorted = devs;
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  kp_ctx *c = new (std::nothrow) kp_ctx();
  if (!c) return KP_ENOMEM;
  c->multi = new (std::nothrow) Multi();
  if (!c->multi) {
    delete c;
    return KP_ENOMEM;
  }
  Multi &M = *c->multi;
  c->device = devs[0];
  c->world = n;
  std::vector<ncclComm_t> comms(n, nullptr);
  // KP_RCCL_SOLO=1 (tests): kp_create_multi([g]) builds its one communicator
  // through ncclCommInitAll too and runs the RCCL exchange on one GPU
  const char *solo_env = knob("KP_RCCL_SOLO");
  const bool solo = n == 1 && solo_env && std::atoi(solo_env) != 0;
  if ((n > 1 || solo) && distinct) {
    if (ncclCommInitAll(comms.data(), n, devs.data()) != ncclSuccess) {
      multi_destroy(c);
      return KP_ERCCL;
    }
    M.rccl = true;
  } else if (n > 1) {
    M.inproc.reset(new InProc());
    M.inproc->n = n;
    M.refs.resize(n);
  }
  int rc = KP_OK;
  for (int i = 0; i < n; ++i) {
    kp_ctx *sh = nullptr;
    const int r = create_one(&sh, devs[i], n, i, nullptr, comms[i], max_pairs);
    if (r != KP_OK) {
      rc = r;
      for (int k = i; k < n; ++k)  // communicators not adopted by a shard
        if (comms[k]) ncclCommDestroy(comms[k]);
      break;
    }
    sh->peer_failed = &M.failed;
    if (M.inproc) {
      M.refs[i] = RankRef{M.inproc.get(), i};
      sh->allgather = inproc_allgather;
      sh->allgather_user = &M.refs[i];
    }
    M.shards.push_back(sh);
  }
  if (rc == KP_OK) {
    try {
      for (int i = 0; i < n; ++i) {
        M.workers.emplace_back(new Worker());
        M.workers.back()->th = std::thread(worker_loop, M.workers.back().get(), devs[i]);
      }
    } catch (...) {
      rc = KP_ENOMEM;
    }
  }
  if (rc != KP_OK) {
    multi_destroy(c);
    return rc;
  }
  *out = c;
  return KP_OK;
}

}  // namespace kp

// raftgpu_rccl.cpp — the built-in RCCL transport for rg_wire_exchange (include/raftgpu.h).
//
// Replicas of a shard live on different GPUs; the per-tick message regions move
// between ranks as one grouped ncclSend / ncclRecv per peer (an all-to-all over xGMI) on the
// transport's own stream, ordered by events after the engine stream's pack and before its unpack:
// pack → transfer → unpack → next tick stay in device order with no host wait, and an engine on
// another stream (the other column half of a rank) keeps computing while the transfer is on the
// wire. The region sizes themselves travel by a small ncclAllGather.
//
// librccl is loaded at run time: a process that already holds an RCCL (PyTorch's, whose file has
// no versioned name) reuses it, otherwise /opt/rocm's librccl.so.1 is opened. Nothing links
// against RCCL, so hosts without multi-GPU needs never load it.
#include <hip/hip_runtime.h>
#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/raftgpu.h"

namespace {

// the slice of rccl.h this file uses (ABI-stable NCCL API; values from /opt/rocm/include/rccl/rccl.h)
typedef struct ncclComm* ncclComm_t;
typedef struct {
  char internal[128];
} ncclUniqueId;
typedef int ncclResult_t;  // ncclSuccess = 0
enum { ncclUint8 = 1, ncclUint64 = 5 };

struct Api {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*Send)(const void*, size_t, int, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void*, size_t, int, int, ncclComm_t, hipStream_t);
  ncclResult_t (*AllGather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*GroupStart)();
  ncclResult_t (*GroupEnd)();
  const char* (*GetErrorString)(ncclResult_t);
  bool ok = false;
};

std::string g_why;

const Api* api() {
  static Api a = [] {
    Api x{};
    void* h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);  // PyTorch's copy, if loaded
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      g_why = std::string("librccl not loadable: ") + dlerror();
      return x;
    }
    auto sym = [&](const char* n) { return dlsym(h, n); };
    x.GetUniqueId = (decltype(x.GetUniqueId))sym("ncclGetUniqueId");
    x.CommInitRank = (decltype(x.CommInitRank))sym("ncclCommInitRank");
    x.CommDestroy = (decltype(x.CommDestroy))sym("ncclCommDestroy");
    x.Send = (decltype(x.Send))sym("ncclSend");
    x.Recv = (decltype(x.Recv))sym("ncclRecv");
    x.AllGather = (decltype(x.AllGather))sym("ncclAllGather");
    x.GroupStart = (decltype(x.GroupStart))sym("ncclGroupStart");
    x.GroupEnd = (decltype(x.GroupEnd))sym("ncclGroupEnd");
    x.GetErrorString = (decltype(x.GetErrorString))sym("ncclGetErrorString");
    x.ok = x.GetUniqueId && x.CommInitRank && x.CommDestroy && x.Send && x.Recv && x.AllGather && x.GroupStart &&
           x.GroupEnd && x.GetErrorString;
    if (!x.ok) g_why = "librccl lacks an expected symbol";
    return x;
  }();
  return a.ok ? &a : nullptr;
}

constexpr uint64_t CHUNK = 256ull << 20;  // bytes per peer per grouped call

struct Rccl {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
  hipStream_t small = nullptr;  // size all-gathers
  hipStream_t xs = nullptr;     // transfers
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  uint64_t* d_sizes = nullptr;  // [2][nranks * 64]
  bool self_rccl = false;       // RAFTGPU_RCCL_SELF=rccl (read at open): the region to self through RCCL too
};

// a failed transfer says why on stderr (the engine only sees the transport's -1)
int why(const Rccl* c, const char* what, int rc = 0) {
  const Api* a = api();
  fprintf(stderr, "raftgpu rccl transport (rank %d of %d): %s%s%s\n", c->rank, c->nranks, what, rc ? ": " : "",
          rc && a ? a->GetErrorString((ncclResult_t)rc) : "");
  return -1;
}

int allgather_u64(void* user, const uint64_t* mine, uint64_t* all, uint32_t n) {
  Rccl* c = (Rccl*)user;
  const Api* a = api();
  if (!a || n > 64) return -1;
  if (hipSetDevice(c->device) != hipSuccess) return -1;
  uint64_t* in = c->d_sizes;
  uint64_t* out = c->d_sizes + 64;
  if (hipMemcpyAsync(in, mine, n * 8ull, hipMemcpyHostToDevice, c->small) != hipSuccess) return -1;
  if (a->AllGather(in, out, n, ncclUint64, c->comm, c->small) != 0) return -1;
  if (hipMemcpyAsync(all, out, (uint64_t)n * c->nranks * 8, hipMemcpyDeviceToHost, c->small) != hipSuccess) return -1;
  return hipStreamSynchronize(c->small) == hipSuccess ? 0 : -1;
}

int alltoallv(void* user, const void* send, const uint64_t* soff, const uint64_t* ssize, void* recv,
              const uint64_t* roff, const uint64_t* rsize, void* stream) {
  Rccl* c = (Rccl*)user;
  const Api* a = api();
  if (!a) return -1;
  hipStream_t st = (hipStream_t)stream, xs = c->xs;
  if (hipSetDevice(c->device) != hipSuccess) return -1;
  if (hipEventRecord(c->ev_in, st) != hipSuccess || hipStreamWaitEvent(xs, c->ev_in, 0) != hipSuccess) return -1;
  // the region to this rank itself is a device copy: RCCL's send/receive to self moved a grown
  // fixed-capacity region at ~25 GB/s (146 ms per step, profiles/r04z_wire_sizing.txt)
  // (RAFTGPU_RCCL_SELF=rccl sends it through RCCL too: the one-rank tests' way to run the grouped path)
  const int me = c->self_rccl ? -1 : c->rank;
  if (me >= 0 && ssize[me] != rsize[me]) {
    char m[160];
    snprintf(m, sizeof m, "the region to itself is %llu bytes sent but %llu received (sizes disagree)",
             (unsigned long long)ssize[me], (unsigned long long)rsize[me]);
    return why(c, m);
  }
  if (me >= 0 && ssize[me] && hipMemcpyAsync((uint8_t*)recv + roff[me], (const uint8_t*)send + soff[me], ssize[me],
                                  hipMemcpyDeviceToDevice, xs) != hipSuccess)
    return -1;
  uint64_t most = 0;
  for (int r = 0; r < c->nranks; ++r)
    if (r != me) most = std::max(most, std::max(ssize[r], rsize[r]));
  // piece k of every region in the k-th group; the two ends of a pair agree on its size, and
  // RCCL matches a pair's sends and receives in issue order, so ranks whose largest region is
  // smaller simply issue fewer groups
  const uint64_t pieces = (most + CHUNK - 1) / CHUNK;
  for (uint64_t k = 0; k < pieces; ++k) {
    if (int rc = a->GroupStart()) return why(c, "ncclGroupStart", rc);
    int bad = 0;  // a failed Send / Recv still closes the group, or every later call on the comm breaks
    for (int r = 0; r < c->nranks && !bad; ++r) {
      if (r == me) continue;
      const uint64_t o = k * CHUNK;
      if (ssize[r] > o)
        bad = a->Send((const uint8_t*)send + soff[r] + o, std::min(CHUNK, ssize[r] - o), ncclUint8, r, c->comm, xs);
      if (!bad && rsize[r] > o)
        bad = a->Recv((uint8_t*)recv + roff[r] + o, std::min(CHUNK, rsize[r] - o), ncclUint8, r, c->comm, xs);
    }
    const int ge = a->GroupEnd();
    if (bad || ge) return why(c, bad ? "ncclSend / ncclRecv" : "ncclGroupEnd", bad ? bad : ge);
  }
  // the engine stream's next work (unpack) waits for the transfers
  if (hipEventRecord(c->ev_out, xs) != hipSuccess || hipStreamWaitEvent(st, c->ev_out, 0) != hipSuccess) return -1;
  return 0;
}

}  // namespace

extern "C" {

int rg_rccl_unique_id(uint8_t id[128]) {
  const Api* a = api();
  if (!a || !id) return RG_EHIP;
  ncclUniqueId u;
  if (a->GetUniqueId(&u) != 0) return RG_EHIP;
  memcpy(id, u.internal, 128);
  return RG_OK;
}

int rg_rccl_open(const uint8_t id[128], int32_t nranks, int32_t rank, int32_t device, rg_transport* out) {
  const Api* a = api();
  if (!a) return RG_EHIP;
  if (!id || !out || nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks) return RG_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return RG_EHIP;
  Rccl* c = new Rccl();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  const char* sv = getenv("RAFTGPU_RCCL_SELF");
  c->self_rccl = sv && !strcmp(sv, "rccl");
  ncclUniqueId u;
  memcpy(u.internal, id, 128);
  if (hipStreamCreateWithFlags(&c->small, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->xs, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming) != hipSuccess ||
      hipMalloc((void**)&c->d_sizes, 2 * 64 * 8 * (uint64_t)nranks) != hipSuccess ||
      a->CommInitRank(&c->comm, nranks, u, rank) != 0) {
    if (c->small) (void)hipStreamDestroy(c->small);
    if (c->xs) (void)hipStreamDestroy(c->xs);
    if (c->ev_in) (void)hipEventDestroy(c->ev_in);
    if (c->ev_out) (void)hipEventDestroy(c->ev_out);
    if (c->d_sizes) (void)hipFree(c->d_sizes);
    delete c;
    return RG_EHIP;
  }
  out->user = c;
  out->allgather_u64 = allgather_u64;
  out->alltoallv = alltoallv;
  return RG_OK;
}

int rg_rccl_close(rg_transport* t) {
  if (!t || !t->user) return RG_EINVAL;
  Rccl* c = (Rccl*)t->user;
  const Api* a = api();
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->small);
  (void)hipStreamSynchronize(c->xs);
  if (a && c->comm) (void)a->CommDestroy(c->comm);
  (void)hipStreamDestroy(c->small);
  (void)hipStreamDestroy(c->xs);
  (void)hipEventDestroy(c->ev_in);
  (void)hipEventDestroy(c->ev_out);
  (void)hipFree(c->d_sizes);
  delete c;
  t->user = nullptr;
  return RG_OK;
}

}  // extern "C"

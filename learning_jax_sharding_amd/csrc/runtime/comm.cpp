// Single-controller RCCL communicators over xGMI (one process drives several
// MI355X; every collective of a device group is issued for all members inside one
// ncclGroupStart/End, each member on its own HIP stream, so one thread cannot deadlock).
//
// A communicator covers an ordered list of DISTINCT physical GPUs (RCCL admits a GPU once
// per communicator; virtual devices sharing a GPU use the framework's copy-based loopback
// backend instead).  Communicators are created with ncclCommInitAll and cached by the Python
// side per device group.  Buffers and streams are passed per member, in member order.
//
// C ABI (ctypes), every call returns 0 or an ncclResult_t / hipError_t code.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#define LJS_RT_API extern "C" __attribute__((visibility("default")))

namespace {

struct Comm {
  std::vector<ncclComm_t> comms;  // one per LOCAL member
  std::vector<int> devs;
  std::vector<int> ranks;         // communicator rank of each local member
  int nranks = 0;                 // ranks in the communicator (all processes)
};

ncclDataType_t to_nccl(int dt) {
  switch (dt) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt32;
    case 4: return ncclInt64;
    case 5: return ncclUint8;
    default: return ncclFloat32;
  }
}

ncclRedOp_t to_op(int op) {
  switch (op) {
    case 1: return ncclMax;
    case 2: return ncclMin;
    case 3: return ncclProd;
    default: return ncclSum;
  }
}

size_t dt_size(int dt) {
  switch (dt) {
    case 1: case 2: return 2;
    case 4: return 8;
    case 5: return 1;
    default: return 4;
  }
}

}  // namespace

LJS_RT_API int ljs_rt_version() { return 1; }

LJS_RT_API int ljs_rt_device_info(int dev, int* out /* cus, lds_bytes, l2_bytes, warp, xcds_hint */,
                                  long* hbm_bytes) {
  hipDeviceProp_t p;
  hipError_t e = hipGetDeviceProperties(&p, dev);
  if (e != hipSuccess) return (int)e;
  out[0] = p.multiProcessorCount;
  out[1] = (int)p.maxSharedMemoryPerMultiProcessor;
  out[2] = p.l2CacheSize;
  out[3] = p.warpSize;
  out[4] = p.multiProcessorCount >= 256 ? 8 : 1;
  *hbm_bytes = (long)p.totalGlobalMem;
  return 0;
}

// handle out; devs = n distinct physical GPU ordinals in member order
LJS_RT_API int ljs_comm_init(int n, const int* devs, void** handle) {
  Comm* c = new Comm();
  c->devs.assign(devs, devs + n);
  c->comms.resize(n);
  ncclResult_t r = ncclCommInitAll(c->comms.data(), n, devs);
  if (r != ncclSuccess) {
    delete c;
    return (int)r;
  }
  for (int i = 0; i < n; ++i) c->ranks.push_back(i);
  c->nranks = n;
  *handle = c;
  return 0;
}

// ---- one process per GPU (torchrun): a communicator with ONE local member, created from a
// unique id that rank 0 publishes through the torch.distributed store.  Collectives are plain
// RCCL calls on the caller's HIP stream, so they are captured into HIP graphs like kernels
// (the training step replays as one graph with its gradient all-reduces inside).
LJS_RT_API int ljs_comm_unique_id_size() { return (int)sizeof(ncclUniqueId); }

LJS_RT_API int ljs_comm_get_unique_id(void* out) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return (int)r;
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

// Restores the caller's current device on scope exit: the helpers below select their device
// with hipSetDevice, which must not leak into the single controller's later calls (torch's
// current_stream() / synchronize() without a device argument act on the current device).
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() { (void)hipGetDevice(&prev); }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

LJS_RT_API int ljs_comm_init_rank(const void* unique_id, int nranks, int rank, int dev, void** handle) {
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return (int)e;
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof(id));
  Comm* c = new Comm();
  c->comms.resize(1);
  ncclResult_t r = ncclCommInitRank(&c->comms[0], nranks, id, rank);
  if (r != ncclSuccess) {
    delete c;
    return (int)r;
  }
  c->devs.push_back(dev);
  c->ranks.push_back(rank);
  c->nranks = nranks;
  *handle = c;
  return 0;
}

// collective over the parent (every rank calls it): ranks with the same colour form one new
// communicator ordered by key; colour < 0 leaves this rank out (*handle = null)
LJS_RT_API int ljs_comm_split_rank(void* parent, int color, int key, void** handle) {
  Comm* p = static_cast<Comm*>(parent);
  if (p->comms.size() != 1) return (int)ncclInvalidUsage;
  ncclComm_t nc = nullptr;
  ncclResult_t r = ncclCommSplit(p->comms[0], color < 0 ? NCCL_SPLIT_NOCOLOR : color, key, &nc, nullptr);
  if (r != ncclSuccess) return (int)r;
  if (color < 0 || nc == nullptr) {
    *handle = nullptr;
    return 0;
  }
  Comm* c = new Comm();
  c->comms.push_back(nc);
  c->devs.push_back(p->devs[0]);
  int rk = 0, n = 0;
  ncclCommUserRank(nc, &rk);
  ncclCommCount(nc, &n);
  c->ranks.push_back(rk);
  c->nranks = n;
  *handle = c;
  return 0;
}

LJS_RT_API int ljs_comm_nranks(void* handle) { return static_cast<Comm*>(handle)->nranks; }

// what RCCL itself reports for a rank communicator (ncclCommCount / ncclCommUserRank / its device),
// not what the caller asked for: the benchmark record's proof that a communicator spans N ranks
LJS_RT_API int ljs_comm_query(void* handle, int* count, int* rank, int* device) {
  Comm* c = static_cast<Comm*>(handle);
  if (c == nullptr || c->comms.size() != 1) return (int)ncclInvalidUsage;
  ncclResult_t r = ncclCommCount(c->comms[0], count);
  if (r != ncclSuccess) return (int)r;
  r = ncclCommUserRank(c->comms[0], rank);
  if (r != ncclSuccess) return (int)r;
  return (int)ncclCommCuDevice(c->comms[0], device);
}

LJS_RT_API int ljs_comm_destroy(void* handle) {
  Comm* c = static_cast<Comm*>(handle);
  for (auto& cm : c->comms) ncclCommDestroy(cm);
  delete c;
  return 0;
}

// in-place capable: sendbufs[i] may equal recvbufs[i]
LJS_RT_API int ljs_comm_all_reduce(void* handle, void* const* sendbufs, void* const* recvbufs, size_t count, int dt,
                                   int op, void* const* streams) {
  Comm* c = static_cast<Comm*>(handle);
  ncclGroupStart();
  for (size_t i = 0; i < c->comms.size(); ++i)
    ncclAllReduce(sendbufs[i], recvbufs[i], count, to_nccl(dt), to_op(op), c->comms[i], (hipStream_t)streams[i]);
  return (int)ncclGroupEnd();
}

// recvbufs[i] holds n * count elements, member-rank-major
LJS_RT_API int ljs_comm_all_gather(void* handle, void* const* sendbufs, void* const* recvbufs, size_t count, int dt,
                                   void* const* streams) {
  Comm* c = static_cast<Comm*>(handle);
  ncclGroupStart();
  for (size_t i = 0; i < c->comms.size(); ++i)
    ncclAllGather(sendbufs[i], recvbufs[i], count, to_nccl(dt), c->comms[i], (hipStream_t)streams[i]);
  return (int)ncclGroupEnd();
}

// sendbufs[i] holds n * count elements (chunk r goes to member r); recv count elements
LJS_RT_API int ljs_comm_reduce_scatter(void* handle, void* const* sendbufs, void* const* recvbufs, size_t count,
                                       int dt, int op, void* const* streams) {
  Comm* c = static_cast<Comm*>(handle);
  ncclGroupStart();
  for (size_t i = 0; i < c->comms.size(); ++i)
    ncclReduceScatter(sendbufs[i], recvbufs[i], count, to_nccl(dt), to_op(op), c->comms[i],
                      (hipStream_t)streams[i]);
  return (int)ncclGroupEnd();
}

// all-to-all of nranks equal chunks of `count` elements: chunk r of rank i lands as chunk i of rank r
LJS_RT_API int ljs_comm_all_to_all(void* handle, void* const* sendbufs, void* const* recvbufs, size_t count, int dt,
                                   void* const* streams) {
  Comm* c = static_cast<Comm*>(handle);
  const size_t n = (size_t)c->nranks;
  const size_t bytes = count * dt_size(dt);
  ncclGroupStart();
  for (size_t i = 0; i < c->comms.size(); ++i) {
    for (size_t r = 0; r < n; ++r) {
      ncclSend(static_cast<const char*>(sendbufs[i]) + r * bytes, count, to_nccl(dt), (int)r, c->comms[i],
               (hipStream_t)streams[i]);
      ncclRecv(static_cast<char*>(recvbufs[i]) + r * bytes, count, to_nccl(dt), (int)r, c->comms[i],
               (hipStream_t)streams[i]);
    }
  }
  return (int)ncclGroupEnd();
}

// point-to-point permutation: pairs (src member, dst member), buffers per pair
LJS_RT_API int ljs_comm_permute(void* handle, int npairs, const int* src, const int* dst, void* const* sendbufs,
                                void* const* recvbufs, size_t count, int dt, void* const* streams) {
  Comm* c = static_cast<Comm*>(handle);
  ncclGroupStart();
  for (int p = 0; p < npairs; ++p) {
    ncclSend(sendbufs[p], count, to_nccl(dt), dst[p], c->comms[src[p]], (hipStream_t)streams[src[p]]);
    ncclRecv(recvbufs[p], count, to_nccl(dt), src[p], c->comms[dst[p]], (hipStream_t)streams[dst[p]]);
  }
  return (int)ncclGroupEnd();
}

LJS_RT_API const char* ljs_comm_error_string(int code) { return ncclGetErrorString((ncclResult_t)code); }

// Sub-communicators by ncclCommSplit of an existing communicator (all members call it inside
// one group): members with the same colour form one new communicator, ranked by key; colour
// < 0 (NCCL_SPLIT_NOCOLOR) leaves a member out.  out_handles[c] receives the communicator of
// colour c (ncolors of them), its members ordered by key.
LJS_RT_API int ljs_comm_split(void* parent, const int* colors, const int* keys, int ncolors, void** out_handles) {
  Comm* p = static_cast<Comm*>(parent);
  const int n = (int)p->comms.size();
  std::vector<ncclComm_t> news(n, nullptr);
  ncclGroupStart();
  for (int i = 0; i < n; ++i) {
    ncclCommSplit(p->comms[i], colors[i] < 0 ? NCCL_SPLIT_NOCOLOR : colors[i], keys[i], &news[i], nullptr);
  }
  ncclResult_t r = ncclGroupEnd();
  if (r != ncclSuccess) return (int)r;
  for (int c = 0; c < ncolors; ++c) {
    Comm* cc = new Comm();
    std::vector<std::pair<int, int>> mem;  // (key, member)
    for (int i = 0; i < n; ++i)
      if (colors[i] == c) mem.push_back({keys[i], i});
    std::sort(mem.begin(), mem.end());
    for (auto& km : mem) {
      cc->comms.push_back(news[km.second]);
      cc->devs.push_back(p->devs[km.second]);
      cc->ranks.push_back((int)cc->ranks.size());
    }
    cc->nranks = (int)cc->comms.size();
    out_handles[c] = cc;
  }
  return 0;
}

// Failure detection: first asynchronous error of any member communicator
// (ncclCommGetAsyncError), 0 when healthy.  ljs_comm_abort tears a wedged communicator down
// so the caller can raise instead of hanging.
LJS_RT_API int ljs_comm_async_error(void* handle) {
  Comm* c = static_cast<Comm*>(handle);
  for (auto& cm : c->comms) {
    ncclResult_t e = ncclSuccess;
    ncclResult_t r = ncclCommGetAsyncError(cm, &e);
    if (r != ncclSuccess) return (int)r;
    if (e != ncclSuccess && e != ncclInProgress) return (int)e;
  }
  return 0;
}

LJS_RT_API int ljs_comm_abort(void* handle) {
  Comm* c = static_cast<Comm*>(handle);
  for (auto& cm : c->comms) ncclCommAbort(cm);
  c->comms.clear();
  return 0;
}

// ---- peer-memory staging buffers for the direct P2P collectives (kernels/p2p.hip)
// fine-grained uncached device memory, zero-filled, with an IPC handle for other processes
LJS_RT_API int ljs_p2p_alloc(int dev, size_t bytes, void** ptr, void* ipc_handle /* 64 bytes or null */) {
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return (int)e;
  e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*ptr, 0, bytes);
  if (e != hipSuccess) return (int)e;
  if (ipc_handle) {
    hipIpcMemHandle_t h;
    e = hipIpcGetMemHandle(&h, *ptr);
    if (e != hipSuccess) return (int)e;
    static_assert(sizeof(h) <= 64, "ipc handle size");
    std::memcpy(ipc_handle, &h, sizeof(h));
  }
  return (int)hipDeviceSynchronize();
}

LJS_RT_API int ljs_p2p_free(void* ptr) { return (int)hipFree(ptr); }

LJS_RT_API int ljs_p2p_open(int dev, const void* ipc_handle, void** ptr) {
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  std::memcpy(&h, ipc_handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

LJS_RT_API int ljs_p2p_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

LJS_RT_API int ljs_p2p_enable_peer(int dev, int peer) {
  if (dev == peer) return 0;
  DeviceGuard guard;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return (int)e;
  e = hipDeviceEnablePeerAccess(peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    return 0;
  }
  return (int)e;
}

LJS_RT_API int ljs_rt_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// capture state of a stream: 0 not capturing, 1 capturing (*id = the capture sequence id, unique
// per capture in this process), < 0 a HIP error.  The p2p groups use it to chain their same-group
// collectives across streams only within one capture (an event recorded outside the capture may
// not be waited on inside it).
LJS_RT_API int ljs_rt_capture_id(void* stream, unsigned long long* id) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long cid = 0;
  hipError_t e = hipStreamGetCaptureInfo(static_cast<hipStream_t>(stream), &st, &cid);
  if (e != hipSuccess) return -(int)e;
  *id = st == hipStreamCaptureStatusActive ? cid : 0;
  return st == hipStreamCaptureStatusActive ? 1 : 0;
}

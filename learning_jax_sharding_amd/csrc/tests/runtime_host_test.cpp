// Host-side test of the native runtime (csrc/runtime/comm.cpp) under AddressSanitizer, on a CPU.
//
// comm.cpp is linked against a HOST MODEL of the RCCL / HIP entry points it calls (defined
// below, not a shim used anywhere else): communicators are heap objects, collectives queued
// between ncclGroupStart/End are executed on host buffers when the outermost group closes, and
// every communicator handed out must be destroyed or aborted exactly once.  That exercises the
// runtime's own logic -- member ordering, split by colour / key, buffer offset arithmetic of
// all-to-all and permute, error propagation, handle lifetimes -- with ASan / LeakSanitizer
// watching every byte it touches (SURVEY §5 "race detection / sanitizers": the GPU side has
// no ASan on this pool; this is the host half).
//
// Build + run: tests/test_runtime_asan.py (host g++ with -fsanitize=address,undefined).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <tuple>
#include <vector>

// ------------------------------------------------------------------ runtime C API under test
extern "C" {
int ljs_rt_version();
int ljs_rt_device_info(int dev, int* out, long* hbm_bytes);
int ljs_comm_init(int n, const int* devs, void** handle);
int ljs_comm_unique_id_size();
int ljs_comm_get_unique_id(void* out);
int ljs_comm_init_rank(const void* unique_id, int nranks, int rank, int dev, void** handle);
int ljs_comm_query(void* handle, int* count, int* rank, int* device);
int ljs_comm_split_rank(void* parent, int color, int key, void** handle);
int ljs_comm_nranks(void* handle);
int ljs_comm_destroy(void* handle);
int ljs_comm_all_reduce(void* handle, void* const* sendbufs, void* const* recvbufs, size_t count, int dt, int op,
                        void* const* streams);
int ljs_comm_all_gather(void* handle, void* const* sendbufs, void* const* recvbufs, size_t count, int dt,
                        void* const* streams);
int ljs_comm_reduce_scatter(void* handle, void* const* sendbufs, void* const* recvbufs, size_t count, int dt, int op,
                            void* const* streams);
int ljs_comm_all_to_all(void* handle, void* const* sendbufs, void* const* recvbufs, size_t count, int dt,
                        void* const* streams);
int ljs_comm_permute(void* handle, int npairs, const int* src, const int* dst, void* const* sendbufs,
                     void* const* recvbufs, size_t count, int dt, void* const* streams);
const char* ljs_comm_error_string(int code);
int ljs_comm_split(void* parent, const int* colors, const int* keys, int ncolors, void** out_handles);
int ljs_comm_async_error(void* handle);
int ljs_comm_abort(void* handle);
int ljs_p2p_alloc(int dev, size_t bytes, void** ptr, void* ipc_handle);
int ljs_p2p_free(void* ptr);
int ljs_p2p_open(int dev, const void* ipc_handle, void** ptr);
int ljs_p2p_close(void* ptr);
int ljs_p2p_enable_peer(int dev, int peer);
int ljs_rt_capture_id(void* stream, unsigned long long* id);
int ljs_rt_ipc_handle_size();
}

// ------------------------------------------------------------------ host model of RCCL
struct ncclComm {
  int world, rank, nranks, dev;
};

namespace {
std::set<ncclComm*> g_live;        // communicators handed out and not yet destroyed
int g_next_world = 1;
int g_group_depth = 0;
int g_fail_init = 0;               // next ncclCommInitAll fails with this result
ncclResult_t g_async = ncclSuccess;
struct Op {
  enum Kind { AR, AG, RS, SEND, RECV, SPLIT } kind;
  const void* send;
  void* recv;
  size_t count;
  ncclDataType_t dt;
  ncclComm_t comm;
  int peer, color, key;
  ncclComm_t* out;
};
std::vector<Op> g_ops;

size_t esize(ncclDataType_t dt) {
  switch (dt) {
    case ncclFloat64: case ncclInt64: case ncclUint64: return 8;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt8: case ncclUint8: return 1;
    default: return 4;
  }
}

ncclComm* make(int world, int rank, int n, int dev) {
  ncclComm* c = new ncclComm{world, rank, n, dev};
  g_live.insert(c);
  return c;
}

void check_live(ncclComm_t c) {
  if (!g_live.count(c)) {
    std::fprintf(stderr, "model: use of a destroyed / unknown communicator\n");
    std::abort();
  }
}

void run_ops() {
  std::vector<Op> ops;
  ops.swap(g_ops);
  // collectives: members of one world issue one op each (float32 sum; others copy)
  std::map<std::pair<int, int>, std::vector<Op*>> coll;  // (world, kind) -> ops
  for (auto& o : ops)
    if (o.kind == Op::AR || o.kind == Op::AG || o.kind == Op::RS) coll[{o.comm->world, (int)o.kind}].push_back(&o);
  for (auto& kv : coll) {
    auto& v = kv.second;
    std::sort(v.begin(), v.end(), [](Op* a, Op* b) { return a->comm->rank < b->comm->rank; });
    const int n = v[0]->comm->nranks;
    if ((int)v.size() != n) {
      std::fprintf(stderr, "model: collective with %zu of %d members in the group\n", v.size(), n);
      std::abort();
    }
    const size_t cnt = v[0]->count, es = esize(v[0]->dt);
    if (kv.first.second == Op::AR) {
      std::vector<float> acc(cnt, 0.f);
      for (Op* o : v)
        for (size_t e = 0; e < cnt; ++e) acc[e] += static_cast<const float*>(o->send)[e];
      for (Op* o : v) std::memcpy(o->recv, acc.data(), cnt * 4);
    } else if (kv.first.second == Op::AG) {
      std::vector<char> all(cnt * es * n);
      for (int r = 0; r < n; ++r) std::memcpy(all.data() + r * cnt * es, v[r]->send, cnt * es);
      for (Op* o : v) std::memcpy(o->recv, all.data(), all.size());
    } else {
      std::vector<float> acc(cnt * n, 0.f);
      for (Op* o : v)
        for (size_t e = 0; e < cnt * n; ++e) acc[e] += static_cast<const float*>(o->send)[e];
      for (int r = 0; r < n; ++r) std::memcpy(v[r]->recv, acc.data() + r * cnt, cnt * 4);
    }
  }
  // point-to-point: the k-th send from a to b pairs with the k-th recv on b from a
  std::map<std::tuple<int, int, int>, std::vector<Op*>> sends, recvs;
  for (auto& o : ops) {
    if (o.kind == Op::SEND) sends[{o.comm->world, o.comm->rank, o.peer}].push_back(&o);
    if (o.kind == Op::RECV) recvs[{o.comm->world, o.peer, o.comm->rank}].push_back(&o);
  }
  for (auto& kv : sends) {
    auto& rv = recvs[kv.first];
    if (rv.size() != kv.second.size()) {
      std::fprintf(stderr, "model: unmatched send / recv\n");
      std::abort();
    }
    for (size_t k = 0; k < rv.size(); ++k)
      std::memcpy(rv[k]->recv, kv.second[k]->send, kv.second[k]->count * esize(kv.second[k]->dt));
  }
  // splits: per (world, colour) ranked by (key, old rank)
  std::map<std::pair<int, int>, std::vector<Op*>> splits;
  for (auto& o : ops)
    if (o.kind == Op::SPLIT) {
      if (o.color < 0) *o.out = nullptr;
      else splits[{o.comm->world, o.color}].push_back(&o);
    }
  for (auto& kv : splits) {
    auto& v = kv.second;
    std::sort(v.begin(), v.end(), [](Op* a, Op* b) {
      return a->key != b->key ? a->key < b->key : a->comm->rank < b->comm->rank;
    });
    const int w = g_next_world++;
    for (size_t i = 0; i < v.size(); ++i) *v[i]->out = make(w, (int)i, (int)v.size(), v[i]->comm->dev);
  }
}

ncclResult_t enqueue(const Op& o) {
  check_live(o.comm);
  g_ops.push_back(o);
  if (g_group_depth == 0) run_ops();
  return ncclSuccess;
}
}  // namespace

extern "C" {
ncclResult_t ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist) {
  if (g_fail_init) {
    ncclResult_t r = (ncclResult_t)g_fail_init;
    g_fail_init = 0;
    return r;
  }
  const int w = g_next_world++;
  for (int i = 0; i < ndev; ++i) comm[i] = make(w, i, ndev, devlist[i]);
  return ncclSuccess;
}
ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  std::memset(id, 0, sizeof(*id));
  const int w = g_next_world++;
  std::memcpy(id, &w, sizeof(w));
  return ncclSuccess;
}
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  int w;
  std::memcpy(&w, &id, sizeof(w));
  *comm = make(w, rank, nranks, 0);
  return ncclSuccess;
}
ncclResult_t ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm, ncclConfig_t*) {
  return enqueue(Op{Op::SPLIT, nullptr, nullptr, 0, ncclFloat32, comm, 0, color, key, newcomm});
}
ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  check_live(comm);
  g_live.erase(comm);
  delete comm;
  return ncclSuccess;
}
ncclResult_t ncclCommAbort(ncclComm_t comm) { return ncclCommDestroy(comm); }
ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  check_live(comm);
  *count = comm->nranks;
  return ncclSuccess;
}
ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  check_live(comm);
  *rank = comm->rank;
  return ncclSuccess;
}
ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* device) {
  check_live(comm);
  *device = comm->dev;
  return ncclSuccess;
}
ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* e) {
  check_live(comm);
  *e = g_async;
  return ncclSuccess;
}
const char* ncclGetErrorString(ncclResult_t) { return "host-model error"; }
ncclResult_t ncclGroupStart() {
  ++g_group_depth;
  return ncclSuccess;
}
ncclResult_t ncclGroupEnd() {
  if (--g_group_depth == 0) run_ops();
  return ncclSuccess;
}
ncclResult_t ncclAllReduce(const void* s, void* r, size_t count, ncclDataType_t dt, ncclRedOp_t, ncclComm_t comm,
                           hipStream_t) {
  return enqueue(Op{Op::AR, s, r, count, dt, comm, 0, 0, 0, nullptr});
}
ncclResult_t ncclAllGather(const void* s, void* r, size_t count, ncclDataType_t dt, ncclComm_t comm, hipStream_t) {
  return enqueue(Op{Op::AG, s, r, count, dt, comm, 0, 0, 0, nullptr});
}
ncclResult_t ncclReduceScatter(const void* s, void* r, size_t count, ncclDataType_t dt, ncclRedOp_t, ncclComm_t comm,
                               hipStream_t) {
  return enqueue(Op{Op::RS, s, r, count, dt, comm, 0, 0, 0, nullptr});
}
ncclResult_t ncclSend(const void* s, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t) {
  return enqueue(Op{Op::SEND, s, nullptr, count, dt, comm, peer, 0, 0, nullptr});
}
ncclResult_t ncclRecv(void* r, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t) {
  return enqueue(Op{Op::RECV, nullptr, r, count, dt, comm, peer, 0, 0, nullptr});
}
}  // extern "C"

// ------------------------------------------------------------------ host model of the HIP calls
namespace {
std::map<void*, size_t> g_allocs;
}
int g_cur_dev = 0;   // the host model's current device
hipError_t hipSetDevice(int d) {
  g_cur_dev = d;
  return hipSuccess;
}
hipError_t hipGetDevice(int* d) {
  *d = g_cur_dev;
  return hipSuccess;
}
hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_t* p, int) {
  std::memset(p, 0, sizeof(*p));
  p->multiProcessorCount = 256;
  p->maxSharedMemoryPerMultiProcessor = 160 << 10;
  p->l2CacheSize = 4 << 20;
  p->warpSize = 64;
  p->totalGlobalMem = 288ull << 30;
  return hipSuccess;
}
hipError_t hipExtMallocWithFlags(void** ptr, size_t bytes, unsigned int) {
  *ptr = std::malloc(bytes);
  g_allocs[*ptr] = bytes;
  return hipSuccess;
}
hipError_t hipMemset(void* dst, int v, size_t bytes) {
  std::memset(dst, v, bytes);
  return hipSuccess;
}
hipError_t hipFree(void* p) {
  if (!g_allocs.erase(p)) return hipErrorInvalidValue;
  std::free(p);
  return hipSuccess;
}
hipError_t hipIpcGetMemHandle(hipIpcMemHandle_t* h, void* p) {
  std::memset(h, 0, sizeof(*h));
  std::memcpy(h, &p, sizeof(p));
  return hipSuccess;
}
hipError_t hipIpcOpenMemHandle(void** p, hipIpcMemHandle_t h, unsigned int) {
  std::memcpy(p, &h, sizeof(*p));
  return hipSuccess;
}
hipError_t hipIpcCloseMemHandle(void*) { return hipSuccess; }
hipError_t hipDeviceSynchronize() { return hipSuccess; }
hipError_t hipDeviceEnablePeerAccess(int, unsigned int) { return hipErrorPeerAccessAlreadyEnabled; }
hipError_t hipGetLastError() { return hipSuccess; }
hipError_t hipStreamGetCaptureInfo(hipStream_t, hipStreamCaptureStatus* st, unsigned long long* id) {
  *st = hipStreamCaptureStatusNone;
  if (id) *id = 0;
  return hipSuccess;
}

// ------------------------------------------------------------------ tests
namespace {
int g_failures = 0;
#define EXPECT(c)                                                          \
  do {                                                                     \
    if (!(c)) {                                                            \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);    \
      ++g_failures;                                                        \
    }                                                                      \
  } while (0)

void test_device_info() {
  int out[5];
  long hbm = 0;
  EXPECT(ljs_rt_device_info(0, out, &hbm) == 0);
  EXPECT(out[0] == 256 && out[1] == 160 * 1024 && out[3] == 64 && out[4] == 8 && hbm == (288l << 30));
  EXPECT(ljs_rt_version() == 1);
}

void test_single_controller_collectives() {
  const int n = 4, devs[n] = {3, 1, 0, 2};
  void* h = nullptr;
  EXPECT(ljs_comm_init(n, devs, &h) == 0);
  EXPECT(ljs_comm_nranks(h) == n);
  const size_t cnt = 5;
  std::vector<std::vector<float>> s(n), r(n);
  void *sp[n], *rp[n], *st[n] = {nullptr, nullptr, nullptr, nullptr};
  // all-reduce (in place on member 0)
  for (int i = 0; i < n; ++i) {
    s[i].assign(cnt, float(i + 1));
    r[i].assign(cnt, -1.f);
    sp[i] = s[i].data();
    rp[i] = i == 0 ? s[i].data() : r[i].data();
  }
  EXPECT(ljs_comm_all_reduce(h, sp, rp, cnt, 0, 0, st) == 0);
  EXPECT(s[0][4] == 10.f && r[3][0] == 10.f);
  // all-gather: member-rank-major
  for (int i = 0; i < n; ++i) {
    s[i].assign(cnt, float(10 * i));
    r[i].assign(cnt * n, -1.f);
    sp[i] = s[i].data();
    rp[i] = r[i].data();
  }
  EXPECT(ljs_comm_all_gather(h, sp, rp, cnt, 0, st) == 0);
  EXPECT(r[2][0] == 0.f && r[2][cnt] == 10.f && r[2][3 * cnt + cnt - 1] == 30.f);
  // reduce-scatter: chunk r of the sum to member r
  for (int i = 0; i < n; ++i) {
    s[i].resize(cnt * n);
    for (size_t e = 0; e < cnt * n; ++e) s[i][e] = float(e / cnt);
    r[i].assign(cnt, -1.f);
    sp[i] = s[i].data();
    rp[i] = r[i].data();
  }
  EXPECT(ljs_comm_reduce_scatter(h, sp, rp, cnt, 0, 0, st) == 0);
  EXPECT(r[0][0] == 0.f && r[3][cnt - 1] == 12.f);
  // all-to-all: chunk j of member i lands as chunk i of member j (exact-size buffers: ASan
  // catches any offset past n * count)
  for (int i = 0; i < n; ++i) {
    for (size_t e = 0; e < cnt * n; ++e) s[i][e] = float(100 * i + e / cnt);
    r[i].assign(cnt * n, -1.f);
    sp[i] = s[i].data();
    rp[i] = r[i].data();
  }
  EXPECT(ljs_comm_all_to_all(h, sp, rp, cnt, 0, st) == 0);
  bool ok = true;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) ok = ok && r[j][i * cnt] == float(100 * i + j);
  EXPECT(ok);
  // permute: a ring shift
  int src[n], dst[n];
  for (int p = 0; p < n; ++p) {
    src[p] = p;
    dst[p] = (p + 1) % n;
    s[p].assign(cnt, float(p));
    r[p].assign(cnt, -1.f);
    sp[p] = s[p].data();
    rp[p] = r[p].data();
  }
  EXPECT(ljs_comm_permute(h, n, src, dst, sp, rp, cnt, 0, st) == 0);
  EXPECT(r[0][0] == 0.f && r[3][cnt - 1] == 3.f);
  // sub-communicators: colours {0, 1, 0, 1}, keys reversing the order inside each colour
  const int colors[n] = {0, 1, 0, 1}, keys[n] = {5, 7, 2, 1};
  void* sub[2] = {nullptr, nullptr};
  EXPECT(ljs_comm_split(h, colors, keys, 2, sub) == 0);
  EXPECT(ljs_comm_nranks(sub[0]) == 2 && ljs_comm_nranks(sub[1]) == 2);
  // member order = key order: colour 0 -> members 2 (key 2), 0 (key 5)
  for (int i = 0; i < 2; ++i) {
    s[i].assign(cnt, float(i + 1));
    r[i].assign(cnt * 2, -1.f);
    sp[i] = s[i].data();
    rp[i] = r[i].data();
  }
  EXPECT(ljs_comm_all_gather(sub[0], sp, rp, cnt, 0, st) == 0);
  EXPECT(r[0][0] == 1.f && r[0][cnt] == 2.f);
  EXPECT(ljs_comm_async_error(sub[1]) == 0);
  g_async = ncclSystemError;
  EXPECT(ljs_comm_async_error(sub[1]) == (int)ncclSystemError);
  g_async = ncclSuccess;
  EXPECT(ljs_comm_abort(sub[1]) == 0);
  EXPECT(ljs_comm_destroy(sub[1]) == 0);  // an aborted handle is still freed exactly once
  EXPECT(ljs_comm_destroy(sub[0]) == 0);
  EXPECT(ljs_comm_destroy(h) == 0);
  EXPECT(std::strlen(ljs_comm_error_string(1)) > 0);
}

void test_init_failure_and_rank_path() {
  g_fail_init = (int)ncclUnhandledCudaError;
  const int devs[2] = {0, 1};
  void* h = reinterpret_cast<void*>(0x1);
  EXPECT(ljs_comm_init(2, devs, &h) == (int)ncclUnhandledCudaError);
  EXPECT(h == reinterpret_cast<void*>(0x1));  // untouched on failure
  // one process per GPU: unique id -> init_rank -> split_rank (NOCOLOR leaves the rank out)
  std::vector<char> id(ljs_comm_unique_id_size());
  EXPECT(ljs_comm_get_unique_id(id.data()) == 0);
  void* r = nullptr;
  EXPECT(ljs_comm_init_rank(id.data(), 1, 0, 0, &r) == 0);
  void* s = reinterpret_cast<void*>(0x1);
  EXPECT(ljs_comm_split_rank(r, -1, 0, &s) == 0 && s == nullptr);
  EXPECT(ljs_comm_split_rank(r, 3, 0, &s) == 0 && s != nullptr && ljs_comm_nranks(s) == 1);
  int qn = -1, qr = -1, qd = -1;   // RCCL's own view (ncclCommCount / UserRank / CuDevice)
  EXPECT(ljs_comm_query(r, &qn, &qr, &qd) == 0 && qn == 1 && qr == 0 && qd == 0);
  EXPECT(ljs_comm_query(s, &qn, &qr, &qd) == 0 && qn == 1 && qr == 0);
  EXPECT(ljs_comm_destroy(s) == 0);
  EXPECT(ljs_comm_destroy(r) == 0);
}

void test_p2p_buffers() {
  void* p = nullptr;
  std::vector<char> ipc(64, 0);
  EXPECT(ljs_rt_ipc_handle_size() <= 64);
  hipSetDevice(3);   // the controller's current device survives every helper below
  EXPECT(ljs_p2p_alloc(0, 4096, &p, ipc.data()) == 0);
  EXPECT(g_cur_dev == 3);
  EXPECT(p != nullptr && static_cast<unsigned char*>(p)[4095] == 0);
  void* q = nullptr;
  EXPECT(ljs_p2p_open(1, ipc.data(), &q) == 0 && q == p);
  EXPECT(g_cur_dev == 3);
  EXPECT(ljs_p2p_close(q) == 0);
  EXPECT(ljs_p2p_enable_peer(0, 1) == 0);  // "already enabled" is success
  EXPECT(g_cur_dev == 3);
  {
    unsigned long long cid = 7;
    EXPECT(ljs_rt_capture_id(nullptr, &cid) == 0 && cid == 0);  // not capturing
  }
  EXPECT(ljs_p2p_free(p) == 0);
}
}  // namespace

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "--asan-selfcheck") == 0) {
    // negative control: the sanitizer must flag this heap overflow (the pytest asserts it does)
    std::vector<float> v(4);
    volatile float* p = v.data();
    return (int)p[argc + 3];
  }
  test_device_info();
  test_single_controller_collectives();
  test_init_failure_and_rank_path();
  test_p2p_buffers();
  if (!g_live.empty()) {
    std::fprintf(stderr, "FAIL: %zu communicators leaked\n", g_live.size());
    ++g_failures;
  }
  if (!g_allocs.empty()) {
    std::fprintf(stderr, "FAIL: %zu peer buffers leaked\n", g_allocs.size());
    ++g_failures;
  }
  std::printf("runtime host test: %s (%d failures)\n", g_failures ? "FAILED" : "ok", g_failures);
  return g_failures ? 1 : 0;
}

// Cross-shard top-k exchange over RCCL (xGMI) for single-process, thread-per-GPU drivers.
//
// The reference gathers every GPU's [Q, k] result to the host and merges with numpy
// (Latest/cuVS-2-gpu/improved_multi_gpu_rag.py:239-277, cuvs-2gpu-main.ipynb:1820-1834); the
// aggregator contract (Attempt_1/test_search_result_aggregator.py:405-457) merges per query.
// Here the per-shard tiles stay on their devices: one grouped ncclAllGather per array (distances,
// ids) over communicators from ncclCommInitAll, then K7 reads the rank-major receive buffer in place
// (MergeArgs::part_stride) on every rank that asks for the result.
//
// RCCL is resolved with dlopen at mivs_comm_init_all, preferring the copy already in the process
// (PyTorch-ROCm links its own librccl.so): two RCCL instances in one process would each bring up
// their own transport state. libmivs.so itself has no link-time dependency on RCCL.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <memory>

#include "capi_util.hpp"
#include "mivs_common.hpp"

using namespace mivs;
using namespace mivs_capi;

namespace {

struct RcclApi {
  void* handle = nullptr;
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  std::string where;
};

template <class F>
void bind(void* h, const char* name, F& fn) {
  fn = reinterpret_cast<F>(dlsym(h, name));
  require(fn != nullptr, std::string("RCCL symbol ") + name + " missing", MIVS_ERR_UNSUPPORTED);
}

const RcclApi& rccl() {
  static std::mutex mu;
  static RcclApi api;
  std::lock_guard<std::mutex> g(mu);
  if (api.handle) return api;
  // already loaded (PyTorch's copy: NEEDED as "librccl.so" by libtorch_hip) first, then the ROCm one
  const char* env = std::getenv("MIVS_RCCL_LIB");
  const char* cands[] = {env, "librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
  void* h = nullptr;
  std::string where;
  for (int pass = 0; pass < 2 && !h; ++pass) {
    for (const char* c : cands) {
      if (!c || !*c) continue;
      h = dlopen(c, RTLD_NOW | RTLD_LOCAL | (pass == 0 ? RTLD_NOLOAD : 0));
      if (h) { where = c; break; }
    }
  }
  require(h != nullptr, std::string("RCCL not found (dlopen librccl.so): ") + (dlerror() ? dlerror() : "?"),
          MIVS_ERR_UNSUPPORTED);
  RcclApi a;
  a.handle = h;
  a.where = where;
  bind(h, "ncclCommInitAll", a.comm_init_all);
  bind(h, "ncclCommDestroy", a.comm_destroy);
  bind(h, "ncclAllGather", a.all_gather);
  bind(h, "ncclGroupStart", a.group_start);
  bind(h, "ncclGroupEnd", a.group_end);
  bind(h, "ncclGetErrorString", a.error_string);
  api = a;
  return api;
}

void ncclchk(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return;
  throw MivsError(MIVS_ERR_HIP, std::string(what) + ": " + rccl().error_string(r));
}

// K7 in gathered mode (k <= kMaxK), or a rank-major -> query-major copy + K8 select (k > kMaxK)
void merge_gathered(const float* gd, const int64_t* gi, int parts, int64_t nq, int k_in, int k, int metric,
                    float* out_d, int64_t* out_i, Buf& tmp, hipStream_t s) {
  if (k <= kMaxK) {
    MergeArgs a{};
    a.in_d = gd;
    a.in_i = gi;
    a.slots_per_q = parts;
    a.part_stride = nq * k_in;
    a.nq = nq;
    a.k_in = k_in;
    a.k = k;
    a.metric = metric;
    a.out_d = out_d;
    a.out_i = out_i;
    HIPCHK(launch_merge(a, s));
    return;
  }
  const size_t n = (size_t)parts * nq * k_in;
  const size_t fb = (n * sizeof(float) + 255) & ~size_t(255);
  tmp.reserve(fb + n * sizeof(int64_t));
  float* td = tmp.as<float>();
  int64_t* ti = reinterpret_cast<int64_t*>(tmp.as<char>() + fb);
  for (int p = 0; p < parts; ++p) {
    HIPCHK(hipMemcpy2DAsync(td + (size_t)p * k_in, sizeof(float) * parts * k_in, gd + (size_t)p * nq * k_in,
                            sizeof(float) * k_in, sizeof(float) * k_in, nq, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpy2DAsync(ti + (size_t)p * k_in, sizeof(int64_t) * parts * k_in, gi + (size_t)p * nq * k_in,
                            sizeof(int64_t) * k_in, sizeof(int64_t) * k_in, nq, hipMemcpyDeviceToDevice, s));
  }
  SelectArgs sa{};
  sa.keys = td;
  sa.ids = ti;
  sa.n_in = (int64_t)parts * k_in;
  sa.nq = nq;
  sa.k = k;
  sa.metric = metric;
  sa.out_d = out_d;
  sa.out_i = out_i;
  HIPCHK(launch_select(sa, s));
}

void check_merge_shape(int parts, int64_t nq, int k_in, int k, int metric) {
  require(k >= 1 && k <= kMaxSelectK, "k must be in [1, " + std::to_string(kMaxSelectK) + "]", MIVS_ERR_UNSUPPORTED);
  require(parts >= 1 && k_in >= 1 && nq >= 0, "bad shape");
  require(metric == MIVS_METRIC_L2 || metric == MIVS_METRIC_IP, "unknown metric");
}

}  // namespace

struct mivs_comm_s {
  std::vector<int> devs;
  std::vector<ncclComm_t> comms;
  // per rank: receive buffers of the two gathers, and the k > 64 transpose scratch
  std::vector<std::unique_ptr<Buf>> recv, tmp;
  // per rank: recorded after the last exchange's reads of recv/tmp; the next exchange's stream waits on it,
  // so a caller that changes streams between calls cannot overwrite a receive buffer still being merged
  std::vector<hipEvent_t> done;
  std::mutex mu;  // one exchange at a time per communicator set (RCCL ops on a comm are ordered)
};

extern "C" {

int32_t mivs_merge_topk_gathered(int32_t device, void* stream, const float* d_in_dist, const int64_t* d_in_ids,
                                 int32_t parts, int64_t nq, int32_t k_in, int32_t k, int32_t metric,
                                 float* d_out_dist, int64_t* d_out_ids) {
  return guarded([&] {
    check_merge_shape(parts, nq, k_in, k, metric);
    if (nq == 0) return;
    require(d_in_dist && d_in_ids && d_out_dist && d_out_ids, "null pointer");
    DeviceGuard dg(device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    Buf tmp;
    merge_gathered(d_in_dist, d_in_ids, parts, nq, k_in, k, metric, d_out_dist, d_out_ids, tmp, s);
    if (tmp.p) HIPCHK(hipStreamSynchronize(s));  // tmp is freed on return
  });
}

int32_t mivs_comm_init_all(int32_t ndev, const int32_t* devs, mivs_comm_t* out) {
  return guarded([&] {
    require(out != nullptr, "null output handle");
    require(ndev >= 1 && devs != nullptr, "ndev must be >= 1");
    int count = 0;
    HIPCHK(hipGetDeviceCount(&count));
    for (int r = 0; r < ndev; ++r) {
      require(devs[r] >= 0 && devs[r] < count, "device " + std::to_string(devs[r]) + " does not exist");
      for (int t = 0; t < r; ++t) require(devs[t] != devs[r], "duplicate device " + std::to_string(devs[r]));
    }
    const RcclApi& api = rccl();
    auto c = std::make_unique<mivs_comm_s>();
    c->devs.assign(devs, devs + ndev);
    c->comms.assign(ndev, nullptr);
    int prev = -1;
    HIPCHK(hipGetDevice(&prev));
    c->done.assign(ndev, nullptr);
    for (int r = 0; r < ndev; ++r) {
      c->recv.emplace_back(new Buf);
      c->tmp.emplace_back(new Buf);
      HIPCHK(hipSetDevice(c->devs[r]));
      HIPCHK(hipEventCreateWithFlags(&c->done[r], hipEventDisableTiming));
    }
    const ncclResult_t rc = api.comm_init_all(c->comms.data(), ndev, c->devs.data());
    (void)hipSetDevice(prev);
    ncclchk(rc, "ncclCommInitAll");
    *out = c.release();
  });
}

int32_t mivs_comm_size(mivs_comm_t comm, int32_t* ndev) {
  return guarded([&] {
    require(comm && ndev, "null argument");
    *ndev = (int32_t)comm->devs.size();
  });
}

int32_t mivs_merge_topk_allgather(mivs_comm_t comm, void* const* streams, const float* const* d_dist,
                                  const int64_t* const* d_ids, int64_t nq, int32_t k_in, int32_t k,
                                  int32_t metric, float* const* d_out_dist, int64_t* const* d_out_ids) {
  return guarded([&] {
    require(comm != nullptr, "null communicator");
    const int P = (int)comm->devs.size();
    check_merge_shape(P, nq, k_in, k, metric);
    require(d_dist && d_ids && d_out_dist && d_out_ids, "null pointer array");
    if (nq == 0) return;
    for (int r = 0; r < P; ++r) {
      require(d_dist[r] && d_ids[r], "rank " + std::to_string(r) + ": null input");
      require((d_out_dist[r] == nullptr) == (d_out_ids[r] == nullptr), "rank " + std::to_string(r) +
              ": give both outputs or neither");
    }
    std::lock_guard<std::mutex> g(comm->mu);
    const RcclApi& api = rccl();
    const size_t per = (size_t)nq * k_in;
    const size_t fbytes = (sizeof(float) * per * P + 255) & ~size_t(255);
    DeviceGuard dg(comm->devs[0]);
    auto stream_of = [&](int r) { return streams ? static_cast<hipStream_t>(streams[r]) : hipStream_t(nullptr); };
    for (int r = 0; r < P; ++r) {  // receive buffers (grow-only; reserve syncs the device if it regrows)
      HIPCHK(hipSetDevice(comm->devs[r]));
      comm->recv[r]->reserve(fbytes + sizeof(int64_t) * per * P);
      HIPCHK(hipStreamWaitEvent(stream_of(r), comm->done[r], 0));
    }
    ncclchk(api.group_start(), "ncclGroupStart");
    for (int r = 0; r < P; ++r) {
      char* base = comm->recv[r]->as<char>();
      const ncclResult_t a = api.all_gather(d_dist[r], base, per, ncclFloat32, comm->comms[r], stream_of(r));
      const ncclResult_t b = a == ncclSuccess
                                 ? api.all_gather(d_ids[r], base + fbytes, per, ncclInt64, comm->comms[r], stream_of(r))
                                 : a;
      if (b != ncclSuccess) {
        (void)api.group_end();
        ncclchk(b, "ncclAllGather");
      }
    }
    ncclchk(api.group_end(), "ncclGroupEnd");
    for (int r = 0; r < P; ++r) {
      HIPCHK(hipSetDevice(comm->devs[r]));
      if (d_out_dist[r]) {
        char* base = comm->recv[r]->as<char>();
        merge_gathered(reinterpret_cast<const float*>(base), reinterpret_cast<const int64_t*>(base + fbytes), P, nq,
                       k_in, k, metric, d_out_dist[r], d_out_ids[r], *comm->tmp[r], stream_of(r));
      }
      HIPCHK(hipEventRecord(comm->done[r], stream_of(r)));
    }
  });
}

void mivs_comm_destroy(mivs_comm_t comm) {
  if (!comm) return;
  {
    std::lock_guard<std::mutex> g(comm->mu);
    int prev = -1;
    (void)hipGetDevice(&prev);
    for (size_t r = 0; r < comm->devs.size(); ++r) {
      (void)hipSetDevice(comm->devs[r]);
      (void)hipDeviceSynchronize();
      if (comm->comms[r]) (void)rccl().comm_destroy(comm->comms[r]);
    }
    for (size_t r = 0; r < comm->devs.size(); ++r) {
      (void)hipSetDevice(comm->devs[r]);
      comm->recv[r].reset();
      comm->tmp[r].reset();
      if (comm->done[r]) (void)hipEventDestroy(comm->done[r]);
    }
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  delete comm;
}

}  // extern "C"

// Framework-owned RCCL communicator: the gradient all-reduce issued straight into librccl on the
// executor's own communication stream, instead of through torch's ProcessGroupNCCL (which re-enqueues every
// collective on its internal stream behind an event and keeps a Work object per call).
//
// One ncclComm_t per process (one rank per GPU, RCCL over xGMI); the 128-B unique id is created on rank 0 and
// shared through the bootstrap process group's object broadcast (parallel/rccl.py).  Every collective is enqueued on
// the calling thread's current HIP stream (torch.cuda.stream context), in place where the op allows it, so the
// caller's events order it against the compute streams exactly like a kernel launch.
//
// The library is the RCCL torch itself loaded (its lib/librccl.so, bound at run time by rccl_load(path)), not a
// link-time librccl: two RCCL copies in one process (torch's and /opt/rocm's share the soname) corrupt each other's
// global state — measured: heap corruption at interpreter exit as soon as both were mapped.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <cstring>
#include <mutex>
#include <string>

namespace {

struct RcclApi {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclGetVersion) GetVersion = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;
  decltype(&ncclCommCuDevice) CommCuDevice = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclBroadcast) Broadcast = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclReduceScatter) ReduceScatter = nullptr;
};
RcclApi g_api;
std::mutex g_api_mu;
bool g_api_ok = false;

template <typename F>
void bind(void* h, F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(h, name));
  TORCH_CHECK(f != nullptr, "RCCL: symbol ", name, " not found");
}

void rccl_load(const std::string& path) {
  std::lock_guard<std::mutex> g(g_api_mu);
  if (g_api_ok) return;
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);   // already mapped by torch: the same handle
  TORCH_CHECK(h != nullptr, "RCCL: cannot open ", path, ": ", dlerror());
  bind(h, g_api.GetUniqueId, "ncclGetUniqueId");
  bind(h, g_api.GetVersion, "ncclGetVersion");
  bind(h, g_api.GetErrorString, "ncclGetErrorString");
  bind(h, g_api.CommInitRank, "ncclCommInitRank");
  bind(h, g_api.CommDestroy, "ncclCommDestroy");
  bind(h, g_api.CommAbort, "ncclCommAbort");
  bind(h, g_api.CommCuDevice, "ncclCommCuDevice");
  bind(h, g_api.AllReduce, "ncclAllReduce");
  bind(h, g_api.Broadcast, "ncclBroadcast");
  bind(h, g_api.AllGather, "ncclAllGather");
  bind(h, g_api.ReduceScatter, "ncclReduceScatter");
  g_api_ok = true;
}

const RcclApi& api() {
  TORCH_CHECK(g_api_ok, "RCCL: library not bound (parallel/rccl.py calls rccl_load with torch's librccl.so)");
  return g_api;
}

#define ncclGetUniqueId api().GetUniqueId
#define ncclGetVersion api().GetVersion
#define ncclGetErrorString api().GetErrorString
#define ncclCommInitRank api().CommInitRank
#define ncclCommDestroy api().CommDestroy
#define ncclCommAbort api().CommAbort
#define ncclCommCuDevice api().CommCuDevice
#define ncclAllReduce api().AllReduce
#define ncclBroadcast api().Broadcast
#define ncclAllGather api().AllGather
#define ncclReduceScatter api().ReduceScatter

#define PVA_RC(x)                                                                                     \
  do {                                                                                                \
    const ncclResult_t r_ = (x);                                                                      \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL: ", #x, " failed: ", ncclGetErrorString(r_));               \
  } while (0)

ncclDataType_t rccl_type(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "RCCL: unsupported dtype ", t.scalar_type());
  }
  return ncclFloat32;
}

ncclRedOp_t rccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "RCCL: unknown reduction '", op, "' (sum, avg, max, min, prod)");
  return ncclSum;
}

hipStream_t cur() { return at::hip::getCurrentHIPStream().stream(); }

void dense(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RCCL ", what, ": contiguous device tensor expected");
}

class RcclComm {
 public:
  RcclComm(const std::string& uid, int64_t nranks, int64_t rank) : nranks_((int)nranks), rank_((int)rank) {
    TORCH_CHECK(uid.size() == sizeof(ncclUniqueId), "RCCL: unique id must be ", sizeof(ncclUniqueId), " bytes");
    TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "RCCL: rank ", rank, " of ", nranks);
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof id);
    PVA_RC(ncclCommInitRank(&comm_, nranks_, id, rank_));
    int dev = -1;
    PVA_RC(ncclCommCuDevice(comm_, &dev));
    device_ = dev;
  }
  ~RcclComm() {
    if (comm_) ncclCommDestroy(comm_);
  }
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  void all_reduce_(const at::Tensor& t, const std::string& op) {
    live();
    dense(t, "all_reduce");
    PVA_RC(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), rccl_type(t), rccl_op(op), comm_, cur()));
  }
  void broadcast_(const at::Tensor& t, int64_t root) {
    live();
    dense(t, "broadcast");
    PVA_RC(ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), rccl_type(t), (int)root, comm_, cur()));
  }
  // out = concat over ranks of `in` (rank order)
  void all_gather(const at::Tensor& out, const at::Tensor& in) {
    live();
    dense(out, "all_gather");
    dense(in, "all_gather");
    TORCH_CHECK(out.scalar_type() == in.scalar_type() && out.numel() == in.numel() * nranks_, "RCCL all_gather: sizes");
    PVA_RC(ncclAllGather(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), rccl_type(in), comm_, cur()));
  }
  // out = this rank's 1/nranks slice of the reduction of `in`
  void reduce_scatter(const at::Tensor& out, const at::Tensor& in, const std::string& op) {
    live();
    dense(out, "reduce_scatter");
    dense(in, "reduce_scatter");
    TORCH_CHECK(out.scalar_type() == in.scalar_type() && in.numel() == out.numel() * nranks_,
                "RCCL reduce_scatter: sizes");
    PVA_RC(ncclReduceScatter(in.data_ptr(), out.data_ptr(), (size_t)out.numel(), rccl_type(in), rccl_op(op), comm_,
                             cur()));
  }
  // tear down without waiting for peers (failure path); the object is unusable afterwards
  void abort() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }
  int rank() const { return rank_; }
  int size() const { return nranks_; }
  int device() const { return device_; }

 private:
  void live() const { TORCH_CHECK(comm_ != nullptr, "RCCL communicator was aborted"); }
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_, device_ = -1;
};

}  // namespace

void register_rccl(pybind11::module& m) {
  m.def("rccl_load", &rccl_load, pybind11::arg("path"));
  m.def("rccl_unique_id", []() {
    ncclUniqueId id;
    PVA_RC(ncclGetUniqueId(&id));
    return pybind11::bytes(reinterpret_cast<const char*>(&id), sizeof id);
  });
  m.def("rccl_version", []() {
    int v = 0;
    PVA_RC(ncclGetVersion(&v));
    return v;
  });
  pybind11::class_<RcclComm>(m, "RcclComm")
      .def(pybind11::init<const std::string&, int64_t, int64_t>(), pybind11::arg("unique_id"), pybind11::arg("nranks"),
           pybind11::arg("rank"))
      .def("all_reduce_", &RcclComm::all_reduce_, pybind11::arg("t"), pybind11::arg("op") = "sum")
      .def("broadcast_", &RcclComm::broadcast_, pybind11::arg("t"), pybind11::arg("root") = 0)
      .def("all_gather", &RcclComm::all_gather, pybind11::arg("out"), pybind11::arg("inp"))
      .def("reduce_scatter", &RcclComm::reduce_scatter, pybind11::arg("out"), pybind11::arg("inp"),
           pybind11::arg("op") = "sum")
      .def("abort", &RcclComm::abort)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def_property_readonly("device", &RcclComm::device);
}

// N06 — RCCL communicator over xGMI, owned by C++.
//
// torch.distributed("nccl") is RCCL too; this direct wrapper exists so the
// governance collectives (X01–X09) can be enqueued on *our* HIP streams and
// captured inside the engine's hipGraphs without a ProcessGroup in the loop.
// The unique id is exchanged by the caller (agent_hypervisor_amd/parallel/rccl.py
// broadcasts it over any torch.distributed group, gloo included).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>

#include "ahv/launch.h"

namespace py = pybind11;

namespace ahv {
namespace host {
namespace {

void check_nccl(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

ncclDataType_t to_dtype(const std::string& s) {
  if (s == "int8") return ncclInt8;
  if (s == "uint8") return ncclUint8;
  if (s == "int32") return ncclInt32;
  if (s == "uint32") return ncclUint32;
  if (s == "int64") return ncclInt64;
  if (s == "uint64") return ncclUint64;
  if (s == "float16") return ncclFloat16;
  if (s == "bfloat16") return ncclBfloat16;
  if (s == "float32") return ncclFloat32;
  if (s == "float64") return ncclFloat64;
  throw std::invalid_argument("unsupported RCCL dtype " + s);
}

ncclRedOp_t to_op(const std::string& s) {
  if (s == "sum") return ncclSum;
  if (s == "prod") return ncclProd;
  if (s == "max") return ncclMax;
  if (s == "min") return ncclMin;
  throw std::invalid_argument("unsupported RCCL reduction " + s);
}

inline void* vp(uintptr_t p) { return reinterpret_cast<void*>(p); }
inline hipStream_t sp(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

class RcclComm {
 public:
  RcclComm(int rank, int world, const py::bytes& uid, int device) : rank_(rank), world_(world), device_(device) {
    std::string raw = uid;
    if (raw.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("bad RCCL unique id length");
    ncclUniqueId id;
    std::memcpy(&id, raw.data(), sizeof(id));
    check_hip(hipSetDevice(device), "hipSetDevice");
    py::gil_scoped_release nogil;
    check_nccl(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
  }
  ~RcclComm() {
    std::unique_lock<std::timed_mutex> lk(mu_);
    if (comm_) ncclCommDestroy(comm_);
  }
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  // Every use of comm_ holds mu_: the watchdog thread may abort while another
  // thread is enqueueing a collective.  abort() raises `abort_req_` first (new
  // issuers then fail fast) and tears the communicator down if it can take the
  // lock; otherwise the issuer inside RCCL aborts on its way out, still holding
  // the lock — ncclCommAbort never runs concurrently with a call on the handle.
  template <class F>
  void issue(const char* what, F&& f) {
    std::unique_lock<std::timed_mutex> lk(mu_);
    if (!comm_ || abort_req_.load()) {
      abort_locked();
      throw std::runtime_error(std::string(what) + ": RCCL communicator was aborted or destroyed");
    }
    const ncclResult_t r = f(comm_);
    if (abort_req_.load()) abort_locked();
    check_nccl(r, what);
  }

  void all_reduce(uintptr_t send, uintptr_t recv, size_t count, const std::string& dt, const std::string& op,
                  uintptr_t stream) {
    const ncclDataType_t t = to_dtype(dt);
    const ncclRedOp_t o = to_op(op);
    issue("ncclAllReduce", [&](ncclComm_t c) { return ncclAllReduce(vp(send), vp(recv), count, t, o, c, sp(stream)); });
  }
  void all_gather(uintptr_t send, uintptr_t recv, size_t count, const std::string& dt, uintptr_t stream) {
    const ncclDataType_t t = to_dtype(dt);
    issue("ncclAllGather", [&](ncclComm_t c) { return ncclAllGather(vp(send), vp(recv), count, t, c, sp(stream)); });
  }
  void reduce_scatter(uintptr_t send, uintptr_t recv, size_t count, const std::string& dt, const std::string& op,
                      uintptr_t stream) {
    const ncclDataType_t t = to_dtype(dt);
    const ncclRedOp_t o = to_op(op);
    issue("ncclReduceScatter",
          [&](ncclComm_t c) { return ncclReduceScatter(vp(send), vp(recv), count, t, o, c, sp(stream)); });
  }
  void broadcast(uintptr_t send, uintptr_t recv, size_t count, const std::string& dt, int root, uintptr_t stream) {
    const ncclDataType_t t = to_dtype(dt);
    issue("ncclBroadcast", [&](ncclComm_t c) { return ncclBroadcast(vp(send), vp(recv), count, t, root, c, sp(stream)); });
  }
  // Point-to-point all-to-all of equal blocks (session re-sharding, P08): block
  // b of `send` goes to rank b, block b of `recv` comes from rank b.
  void all_to_all(uintptr_t send, uintptr_t recv, size_t block_count, const std::string& dt, size_t elem_bytes,
                  uintptr_t stream) {
    const ncclDataType_t t = to_dtype(dt);
    const size_t stride = block_count * elem_bytes;
    issue("ncclAllToAll", [&](ncclComm_t c) {
      ncclResult_t r = ncclGroupStart();
      for (int k = 0; r == ncclSuccess && k < world_; ++k) {
        r = ncclSend(static_cast<char*>(vp(send)) + k * stride, block_count, t, k, c, sp(stream));
        if (r == ncclSuccess) r = ncclRecv(static_cast<char*>(vp(recv)) + k * stride, block_count, t, k, c, sp(stream));
      }
      const ncclResult_t e = ncclGroupEnd();
      return r != ncclSuccess ? r : e;
    });
  }
  void destroy() {
    std::unique_lock<std::timed_mutex> lk(mu_);
    if (comm_) {
      const ncclResult_t r = ncclCommDestroy(comm_);
      comm_ = nullptr;
      check_nccl(r, "ncclCommDestroy");
    }
  }
  // Asynchronous error state of the communicator (failure detection, §5.3):
  // "" while healthy, else RCCL's error text ("busy" if an enqueue held the lock
  // for over a second — the caller polls again).
  std::string async_error() {
    std::unique_lock<std::timed_mutex> lk(mu_, std::defer_lock);
    if (!lk.try_lock_for(std::chrono::seconds(1))) return "busy";
    if (!comm_) return abort_req_.load() ? "aborted" : "destroyed";
    ncclResult_t st = ncclSuccess;
    check_nccl(ncclCommGetAsyncError(comm_, &st), "ncclCommGetAsyncError");
    return st == ncclSuccess || st == ncclInProgress ? std::string() : std::string(ncclGetErrorString(st));
  }
  // Tear down a communicator whose peers may be gone; pending collectives are
  // cancelled instead of waited for.  Safe from any thread (see issue()).
  void abort() {
    abort_req_.store(true);
    std::unique_lock<std::timed_mutex> lk(mu_, std::defer_lock);
    if (lk.try_lock_for(std::chrono::seconds(2))) abort_locked();
  }
  bool aborted() const { return abort_req_.load(); }
  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }

 private:
  void abort_locked() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }
  ncclComm_t comm_ = nullptr;
  std::timed_mutex mu_;
  std::atomic<bool> abort_req_{false};
  int rank_, world_, device_;
};

}  // namespace

static std::string so_of(const void* sym) {
  Dl_info info{};
  if (dladdr(sym, &info) && info.dli_fname) return info.dli_fname;
  return "?";
}

void register_comm(py::module_& m) {
  m.def(
      "runtime_libraries",
      []() {
        py::dict d;
        d["hip"] = so_of(reinterpret_cast<const void*>(&hipGetDeviceCount));
        d["rccl"] = so_of(reinterpret_cast<const void*>(&ncclGetUniqueId));
        return d;
      },
      "Paths of the shared objects that provide HIP and RCCL to this extension "
      "(they must be the ones torch loaded).");
  m.def("rccl_unique_id", []() {
    ncclUniqueId id;
    check_nccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
  });
  m.def("rccl_version", []() {
    int v = 0;
    check_nccl(ncclGetVersion(&v), "ncclGetVersion");
    return v;
  });
  py::class_<RcclComm, std::unique_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init<int, int, const py::bytes&, int>(), py::arg("rank"), py::arg("world"), py::arg("unique_id"),
           py::arg("device"))
      .def("all_reduce", &RcclComm::all_reduce, py::call_guard<py::gil_scoped_release>())
      .def("all_gather", &RcclComm::all_gather, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &RcclComm::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("all_to_all", &RcclComm::all_to_all, py::call_guard<py::gil_scoped_release>())
      .def("destroy", &RcclComm::destroy)
      .def("async_error", &RcclComm::async_error, py::call_guard<py::gil_scoped_release>())
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("aborted", &RcclComm::aborted)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("device", &RcclComm::device);
}

}  // namespace host
}  // namespace ahv

// Python bindings of the native runtime (module ddlb_amd._C).
//
// Tensors cross the boundary as raw device pointers + the caller's HIP stream handle
// (torch.cuda.current_stream().cuda_stream): no dependency on torch's C++ ABI, and every call is a
// single C++ entry. Python-side wrappers (ddlb_amd/ops, ddlb_amd/parallel) validate shapes, dtypes,
// devices and alignment BEFORE anything is launched. Symmetric buffers are exported to torch via
// DLPack (kDLROCM) so they can be used as ordinary tensors.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <ATen/dlpack.h>

#include <memory>
#include <tuple>

#include "comm/comm.h"
#include "gemm/gemm.h"
#include "runtime/kernels.h"
#include "runtime/plan.h"

namespace py = pybind11;
using namespace ddlb;

namespace {

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    (void)hipGetLastError();  // keep torch's next error check clean
    throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
  }
}

struct DLCtx {
  std::shared_ptr<void> owner;  // keeps the allocation (symmetric buffer / RCCL memory) alive
  int64_t shape[1];
};

void dl_deleter(DLManagedTensor* t) {
  delete static_cast<DLCtx*>(t->manager_ctx);
  delete t;
}

void capsule_destructor(PyObject* cap) {
  if (PyCapsule_IsValid(cap, "dltensor")) {  // never consumed
    auto* t = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
    if (t && t->deleter) t->deleter(t);
  }
}

py::object raw_dlpack(std::shared_ptr<void> owner, uintptr_t ptr, size_t bytes, int device) {
  auto* ctx = new DLCtx{std::move(owner), {(int64_t)bytes}};
  auto* t = new DLManagedTensor();
  t->dl_tensor.data = (void*)ptr;
  t->dl_tensor.device = DLDevice{kDLROCM, device};
  t->dl_tensor.ndim = 1;
  t->dl_tensor.dtype = DLDataType{kDLUInt, 8, 1};
  t->dl_tensor.shape = ctx->shape;
  t->dl_tensor.strides = nullptr;
  t->dl_tensor.byte_offset = 0;
  t->manager_ctx = ctx;
  t->deleter = dl_deleter;
  return py::reinterpret_steal<py::object>(PyCapsule_New(t, "dltensor", capsule_destructor));
}

py::object buffer_dlpack(std::shared_ptr<SymmetricBuffer> buf, int device) {
  return raw_dlpack(buf, buf->local(), buf->bytes(), device);
}

// CU holder of the rccl_cap preflight phase (ddlb_amd/parallel/preflight.py): holds n CUs with
// hold_cus_kernel while a capped RCCL collective must finish beside them. The counters live in
// host-coherent pinned memory, so the host sees residency and releases the holders without any
// stream ordering (the collective is queued on another stream).
class CuHolder {
 public:
  explicit CuHolder(int device) : device_(device) {
    check(hipSetDevice(device), "hipSetDevice");
    check(hipHostMalloc((void**)&host_, 512, hipHostMallocCoherent | hipHostMallocMapped),
          "hipHostMalloc");
    check(hipHostGetDevicePointer((void**)&dev_, host_, 0), "hipHostGetDevicePointer");
    reset();
  }
  ~CuHolder() {
    if (host_) {
      release();
      hipSetDevice(device_);
      hipDeviceSynchronize();
      hipHostFree(host_);
    }
  }
  void start(int nwg, uintptr_t stream, double max_s) {
    reset();
    HoldArgs a;
    a.arrived = dev_;
    a.go = dev_ + 32;
    a.timeout_word = dev_ + 64;
    a.max_ticks = (uint64_t)(max_s * 1e8);  // s_memrealtime: 100 MHz
    check(hipSetDevice(device_), "hipSetDevice");
    check(hold_cus_launch(a, nwg, (hipStream_t)stream), "hold_cus_launch");
  }
  unsigned arrived() const { return __atomic_load_n(host_, __ATOMIC_ACQUIRE); }
  unsigned timeout_bits() const { return __atomic_load_n(host_ + 64, __ATOMIC_ACQUIRE); }
  void release() { __atomic_store_n(host_ + 32, 1u, __ATOMIC_RELEASE); }

 private:
  void reset() {
    __atomic_store_n(host_, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(host_ + 32, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(host_ + 64, 0u, __ATOMIC_RELEASE);
  }
  int device_;
  unsigned* host_ = nullptr;  // [0] arrived, [32] go, [64] timeout bits (separate 128-B lines)
  unsigned* dev_ = nullptr;
};

GemmArgs make_args(uintptr_t a, uintptr_t b, uintptr_t c, int64_t lda, int64_t ldb, int64_t ldc,
                   int M, int N, int K, int64_t a_grp, int64_t a_gstride, int64_t c_grp,
                   int64_t c_gstride) {
  GemmArgs g;
  g.a = (const void*)a; g.b = (const void*)b; g.c = (void*)c;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K;
  g.a_grp = a_grp; g.a_gstride = a_gstride; g.c_grp = c_grp; g.c_gstride = c_gstride;
  return g;
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "ddlb_amd native runtime: CDNA4 MFMA GEMM, RCCL/IPC data plane, plan executor";
  m.attr("OP_WORDS") = kOpWords;
  m.attr("MAX_REDUCE_SRC") = kMaxReduceSrc;
  m.attr("MAX_COPY_SEG") = kMaxCopySeg;
  m.attr("MAX_SIGNAL") = kMaxSignal;

  m.def("gemm",
        [](uintptr_t a, uintptr_t b, uintptr_t c, int64_t lda, int64_t ldb, int64_t ldc, int M,
           int N, int K, int din, int dout, int tile, int mode, int64_t a_grp, int64_t a_gstride,
           int64_t c_grp, int64_t c_gstride, uintptr_t stream, int act, int ksplit) {
          GemmArgs g = make_args(a, b, c, lda, ldb, ldc, M, N, K, a_grp, a_gstride, c_grp,
                                 c_gstride);
          g.act = act;
          g.ksplit = ksplit > 1 ? ksplit : 1;
          check(gemm_launch(g, din, dout, tile, mode, (hipStream_t)stream), "gemm_launch");
        },
        py::arg("a"), py::arg("b"), py::arg("c"), py::arg("lda"), py::arg("ldb"), py::arg("ldc"),
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("din"), py::arg("dout"),
        py::arg("tile") = 0, py::arg("mode") = 0, py::arg("a_grp") = 0, py::arg("a_gstride") = 0,
        py::arg("c_grp") = 0, py::arg("c_gstride") = 0, py::arg("stream") = 0,
        py::arg("act") = 0, py::arg("ksplit") = 1);
  m.def("gemm_fast_path_ok",
        [](uintptr_t a, uintptr_t b, uintptr_t c, int64_t lda, int64_t ldb, int64_t ldc, int M,
           int N, int K, int din, int dout) {
          GemmArgs g = make_args(a, b, c, lda, ldb, ldc, M, N, K, M, M, M, M);
          return gemm_fast_path_ok(g, din, dout);
        });
  m.def("choose_tile", &choose_tile);
  m.def("tile_rows", &tile_rows);
  m.def("tile_cols", &tile_cols);

  m.def("reduce_sum",
        [](uintptr_t dst, std::vector<uintptr_t> srcs, int64_t count, int dtype, uintptr_t s,
           int src_dtype) {
          ReduceArgs a;
          a.dst = (void*)dst;
          a.count = count;
          a.nsrc = (int)srcs.size();
          if (a.nsrc < 1 || a.nsrc > kMaxReduceSrc) throw std::runtime_error("1..16 sources");
          for (int i = 0; i < a.nsrc; ++i) a.src[i] = (const void*)srcs[(size_t)i];
          check(reduce_sum_launch(a, dtype, (hipStream_t)s, src_dtype), "reduce_sum");
        },
        py::arg("dst"), py::arg("srcs"), py::arg("count"), py::arg("dtype"), py::arg("stream"),
        py::arg("src_dtype") = -1);
  m.def("copy",
        [](uintptr_t dst, uintptr_t src, int64_t bytes, int max_blocks, uintptr_t s) {
          CopyArgs a;
          a.nseg = 1;
          a.dst[0] = (void*)dst;
          a.src[0] = (const void*)src;
          a.bytes[0] = bytes;
          check(copy_launch(a, max_blocks, (hipStream_t)s), "copy");
        });
  m.def("memcpy_async",  // one copy-engine copy (diagnostics: the xGMI probe's SDMA pulls)
        [](uintptr_t dst, uintptr_t src, int64_t bytes, uintptr_t s) {
          check(hipMemcpyAsync((void*)dst, (const void*)src, (size_t)bytes,
                               hipMemcpyDeviceToDevice, (hipStream_t)s),
                "hipMemcpyAsync");
        });
  m.def("copy_multi",  // segments (dst, src, bytes) copied concurrently by one CU kernel
        [](std::vector<std::tuple<uintptr_t, uintptr_t, int64_t>> segs, int max_blocks,
           uintptr_t s) {
          CopyArgs a;
          a.nseg = (int)segs.size();
          if (a.nseg < 1 || a.nseg > kMaxCopySeg) throw std::runtime_error("1..8 segments");
          for (int i = 0; i < a.nseg; ++i) {
            a.dst[i] = (void*)std::get<0>(segs[(size_t)i]);
            a.src[i] = (const void*)std::get<1>(segs[(size_t)i]);
            a.bytes[i] = std::get<2>(segs[(size_t)i]);
          }
          check(copy_launch(a, max_blocks, (hipStream_t)s), "copy_multi");
        });
  m.def("copy_batch_api_available", &copy_batch_api_available);
  m.def("copy_batch_status", &copy_batch_status);
  m.def("copy_batch",  // copy-engine copies (dst, src, bytes) submitted as one batch
        [](std::vector<std::tuple<uintptr_t, uintptr_t, int64_t>> segs, uintptr_t s) {
          std::vector<void*> d, sr;
          std::vector<size_t> b;
          for (auto& t : segs) {
            d.push_back((void*)std::get<0>(t));
            sr.push_back((void*)std::get<1>(t));
            b.push_back((size_t)std::get<2>(t));
          }
          if (d.empty()) return;
          check(copy_batch(d.data(), sr.data(), b.data(), d.size(), (hipStream_t)s), "copy_batch");
        });
  m.def("install_crash_handler", &install_crash_handler);
  m.def("device_synchronize", []() { check(hipDeviceSynchronize(), "hipDeviceSynchronize"); });
  m.def("get_last_error", []() { return std::string(hipGetErrorString(hipGetLastError())); });

  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def_static("unique_id", []() { return py::bytes(RcclComm::unique_id()); })
      // (the id arrives as std::string: converted from bytes before the GIL is released)
      .def(py::init([](const std::string& uid, int nranks, int rank, int device, int max_ctas) {
             return std::make_shared<RcclComm>(uid, nranks, rank, device, max_ctas);
           }),
           py::arg("uid"), py::arg("nranks"), py::arg("rank"), py::arg("device"),
           py::arg("max_ctas") = 0, py::call_guard<py::gil_scoped_release>())
      .def("destroy", &RcclComm::destroy)
      // collectives on the caller's stream (preflight / diagnostics: the plans go through the
      // executor); count in elements of dtype (DT_* codes)
      .def("all_gather",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, uintptr_t s) {
             DDLB_NCCL(ncclAllGather((const void*)send, (void*)recv, count, nccl_dtype(dtype),
                                     c.get(), (hipStream_t)s));
           })
      .def("reduce_scatter",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, uintptr_t s) {
             DDLB_NCCL(ncclReduceScatter((const void*)send, (void*)recv, count, nccl_dtype(dtype),
                                         ncclSum, c.get(), (hipStream_t)s));
           })
      .def("async_error", &RcclComm::async_error)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("max_ctas", &RcclComm::max_ctas);
  py::class_<CuHolder>(m, "CuHolder")
      .def(py::init<int>(), py::arg("device"))
      .def("start", &CuHolder::start, py::arg("nwg"), py::arg("stream"),
           py::arg("max_s") = 10.0)
      .def("arrived", &CuHolder::arrived)
      .def("timeout_bits", &CuHolder::timeout_bits)
      .def("release", &CuHolder::release);

  py::class_<RcclMem, std::shared_ptr<RcclMem>>(m, "RcclMem")
      .def(py::init<std::shared_ptr<RcclComm>, size_t, int>(), py::arg("comm"), py::arg("bytes"),
           py::arg("device"))
      .def("release", &RcclMem::release)
      .def("local", &RcclMem::local)
      .def_property_readonly("registered", &RcclMem::registered)
      .def_property_readonly("bytes", &RcclMem::bytes);
  m.def("rccl_mem_dlpack", [](std::shared_ptr<RcclMem> b, int device) {
    return raw_dlpack(b, b->local(), b->bytes(), device);
  });

  py::class_<SymmetricBuffer, std::shared_ptr<SymmetricBuffer>>(m, "SymmetricBuffer")
      .def(py::init<size_t, int, bool>(), py::arg("bytes"), py::arg("device"),
           py::arg("uncached") = false)
      .def_property_readonly("uncached", &SymmetricBuffer::uncached)
      .def("ipc_handle", [](const SymmetricBuffer& b) { return py::bytes(b.ipc_handle()); })
      .def("open_peers",
           [](SymmetricBuffer& b, std::vector<py::bytes> hs, int my_rank) {
             std::vector<std::string> v;
             for (auto& h : hs) v.emplace_back(std::string(h));
             b.open_peers(v, my_rank);
           })
      .def("close_peers", &SymmetricBuffer::close_peers)
      .def("release", &SymmetricBuffer::release)
      .def("local", &SymmetricBuffer::local)
      .def("peer", &SymmetricBuffer::peer)
      .def("npeers", &SymmetricBuffer::npeers)
      .def_property_readonly("bytes", &SymmetricBuffer::bytes);
  m.def("buffer_dlpack", &buffer_dlpack);

  py::class_<PlanExecutor, std::shared_ptr<PlanExecutor>>(m, "PlanExecutor")
      .def(py::init<int, int, int, const std::vector<int>&>())
      .def("load", &PlanExecutor::load)
      .def("set_comm", [](PlanExecutor& p, std::shared_ptr<RcclComm> c) { p.set_comm(c.get()); },
           py::keep_alive<1, 2>())
      .def("run", &PlanExecutor::run)
      .def("epoch", &PlanExecutor::epoch)
      .def("nops", &PlanExecutor::nops)
      .def("stream", &PlanExecutor::stream)
      .def("timeout_word", &PlanExecutor::timeout_word)
      .def("read_timeout", &PlanExecutor::read_timeout)
      .def("enable_graph", &PlanExecutor::enable_graph)
      .def("graph_enabled", &PlanExecutor::graph_enabled)
      .def("graph_capturable", &PlanExecutor::graph_capturable)
      .def("set_timeline", &PlanExecutor::set_timeline)
      .def("timeline", &PlanExecutor::timeline)
      .def("host_times", &PlanExecutor::host_times)
      .def("set_cu_split", &PlanExecutor::set_cu_split)
      .def("cu_split", &PlanExecutor::cu_split)
      .def("stream_info", &PlanExecutor::stream_info)
      .def("set_trace", &PlanExecutor::set_trace);
}

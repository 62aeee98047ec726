// RCCL communicator and HIP IPC symmetric buffers (see comm.h).
//
// Replaces the reference's NCCL/UCC process-group data plane (ddlb/primitives/*/pytorch.py:53-59)
// and nvFuser's CommunicatorBackend.cuda symmetric memory (TPColumnwise/fuser.py:44-45,131-132).
#include "comm.h"

#include <cstring>

#include "../gemm/gemm.h"

namespace ddlb {

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  DDLB_NCCL(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(const std::string& uid, int nranks, int rank, int device, int max_ctas)
    : rank_(rank), nranks_(nranks), max_ctas_(max_ctas > 0 ? max_ctas : 0) {
  if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  DDLB_HIP(hipSetDevice(device));
  if (max_ctas_ == 0) {
    DDLB_NCCL(ncclCommInitRank(&comm_, nranks, id, rank));
    return;
  }
  // The CTA cap is a communicator attribute (the layout up to maxCTAs is the same in every
  // ncclConfig_t version); minCTAs is lowered with it so the pair stays valid. A library that
  // refuses the config fails loudly: a capped communicator is a safety property, never a hint.
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.maxCTAs = max_ctas_;
  cfg.minCTAs = 1;
  DDLB_NCCL(ncclCommInitRankConfig(&comm_, nranks, id, rank, &cfg));
}

RcclComm::~RcclComm() {
  try {
    destroy();
  } catch (...) {
  }
}

void RcclComm::destroy() {
  if (comm_ != nullptr) {
    ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
}

std::string RcclComm::async_error() const {
  if (comm_ == nullptr) return "";
  ncclResult_t r = ncclSuccess;
  ncclCommGetAsyncError(comm_, &r);
  return r == ncclSuccess ? std::string() : std::string(ncclGetErrorString(r));
}

ncclDataType_t nccl_dtype(int dt) {
  switch (dt) {
    case DT_F32: return ncclFloat32;
    case DT_F16: return ncclFloat16;
    case DT_BF16: return ncclBfloat16;
    case DT_F64: return ncclFloat64;
    case DT_FP8: case DT_U8: return ncclUint8;  // moved as bytes (no fp8 reductions needed)
    default: throw std::runtime_error("unsupported dtype for RCCL");
  }
}

RcclMem::RcclMem(std::shared_ptr<RcclComm> comm, size_t bytes, int device)
    : comm_(std::move(comm)), bytes_(bytes ? bytes : 256), device_(device) {
  if (!comm_ || comm_->get() == nullptr) throw std::runtime_error("RcclMem: no communicator");
  DDLB_HIP(hipSetDevice(device));
  DDLB_NCCL(ncclMemAlloc(&ptr_, bytes_));
  DDLB_HIP(hipMemset(ptr_, 0, bytes_));
  DDLB_HIP(hipDeviceSynchronize());
  const ncclResult_t r = ncclCommRegister(comm_->get(), ptr_, bytes_, &handle_);
  if (r != ncclSuccess) {
    ncclMemFree(ptr_);
    ptr_ = nullptr;
    throw std::runtime_error(std::string("ncclCommRegister: ") + ncclGetErrorString(r));
  }
}

RcclMem::~RcclMem() {
  try {
    release();
    if (ptr_ != nullptr) {
      hipSetDevice(device_);
      hipDeviceSynchronize();
      ncclMemFree(ptr_);
      ptr_ = nullptr;
    }
  } catch (...) {
  }
}

// Deregister from the communicator now (it may be destroyed right after); the memory itself is
// freed by the destructor, i.e. when the last owner goes — DLPack views handed to torch (e.g.
// a rowwise plan's output slice returned by run()) hold one, so they stay valid after close().
void RcclMem::release() {
  if (ptr_ == nullptr || handle_ == nullptr) return;
  hipSetDevice(device_);
  hipDeviceSynchronize();
  if (comm_ && comm_->get() != nullptr) ncclCommDeregister(comm_->get(), handle_);
  handle_ = nullptr;
}

SymmetricBuffer::SymmetricBuffer(size_t bytes, int device, bool uncached)
    : bytes_(bytes), device_(device), uncached_(uncached) {
  DDLB_HIP(hipSetDevice(device));
  if (uncached)
    DDLB_HIP(hipExtMallocWithFlags(&ptr_, bytes ? bytes : 256, hipDeviceMallocUncached));
  else
    DDLB_HIP(hipMalloc(&ptr_, bytes ? bytes : 256));
  DDLB_HIP(hipMemset(ptr_, 0, bytes ? bytes : 256));
  DDLB_HIP(hipDeviceSynchronize());
}

SymmetricBuffer::~SymmetricBuffer() { release(); }

void SymmetricBuffer::release() {
  close_peers();
  if (ptr_ != nullptr) {
    hipDeviceSynchronize();
    hipFree(ptr_);
    ptr_ = nullptr;
    (void)hipGetLastError();
  }
}

std::string SymmetricBuffer::ipc_handle() const {
  hipIpcMemHandle_t h;
  DDLB_HIP(hipIpcGetMemHandle(&h, ptr_));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void SymmetricBuffer::open_peers(const std::vector<std::string>& handles, int my_rank) {
  close_peers();
  peers_.assign(handles.size(), nullptr);
  opened_.assign(handles.size(), false);
  for (size_t r = 0; r < handles.size(); ++r) {
    if ((int)r == my_rank) {
      peers_[r] = ptr_;
      continue;
    }
    if (handles[r].size() != sizeof(hipIpcMemHandle_t))
      throw std::runtime_error("bad IPC handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[r].data(), sizeof(h));
    void* p = nullptr;
    DDLB_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    peers_[r] = p;
    opened_[r] = true;
  }
}

void SymmetricBuffer::close_peers() {
  for (size_t r = 0; r < peers_.size(); ++r)
    if (opened_[r] && peers_[r] != nullptr) hipIpcCloseMemHandle(peers_[r]);
  peers_.clear();
  opened_.clear();
}

}  // namespace ddlb

// Native data plane: our own RCCL communicator + HIP IPC symmetric memory.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace ddlb {

#define DDLB_HIP(x)                                                                       \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      (void)hipGetLastError(); /* do not leave a stale error for torch's next check */    \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + ": " #x);      \
    }                                                                                     \
  } while (0)
#define DDLB_NCCL(x)                                                                       \
  do {                                                                                     \
    ncclResult_t r_ = (x);                                                                 \
    if (r_ != ncclSuccess)                                                                 \
      throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(r_) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + ": " #x);       \
  } while (0)

// RCCL communicator created from a unique id that Python exchanges over the torch store, so the
// collectives are enqueued on *our* HIP streams (not torch's internal NCCL stream).
class RcclComm {
 public:
  static std::string unique_id();  // 128 raw bytes
  // max_ctas > 0: the communicator's kernels launch at most that many workgroups (ncclConfig_t
  // maxCTAs, one workgroup per channel). A flag-gated persistent GEMM fed by this communicator's
  // collectives leaves `reserve_cus` CUs free; with max_ctas <= reserve_cus the collective can
  // always be resident beside the spinning tiles (ddlb_amd/parallel/algorithms.py).
  RcclComm(const std::string& uid, int nranks, int rank, int device, int max_ctas = 0);
  ~RcclComm();
  void destroy();
  ncclComm_t get() const { return comm_; }
  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  int max_ctas() const { return max_ctas_; }
  std::string async_error() const;

 private:
  ncclComm_t comm_ = nullptr;
  int rank_ = 0, nranks_ = 1, max_ctas_ = 0;
};

ncclDataType_t nccl_dtype(int dt);  // DT_* -> ncclDataType_t

// A buffer RCCL may use zero-copy: allocated with ncclMemAlloc and registered with the
// communicator (ncclCommRegister), the analogue of nvFuser's symmetric-memory allocations
// (reference TPColumnwise/fuser.py:44-45). release() deregisters it while the communicator lives;
// the memory is freed (ncclMemFree) when the last owner, e.g. a DLPack view, lets go.
class RcclMem {
 public:
  RcclMem(std::shared_ptr<RcclComm> comm, size_t bytes, int device);
  ~RcclMem();
  void release();
  uintptr_t local() const { return (uintptr_t)ptr_; }
  size_t bytes() const { return bytes_; }
  bool registered() const { return handle_ != nullptr; }

 private:
  std::shared_ptr<RcclComm> comm_;
  void* ptr_ = nullptr;
  void* handle_ = nullptr;
  size_t bytes_ = 0;
  int device_ = 0;
};

// One symmetric allocation: a hipMalloc'd buffer on this device + the IPC-mapped pointers of the
// same-named buffer on every peer (index = rank; own rank -> local pointer).
class SymmetricBuffer {
 public:
  // uncached: fine-grained, never cached in any GPU's L2 (hipDeviceMallocUncached). Used for the
  // cross-process flag words: peers write them over xGMI while this GPU's command processor or a
  // kernel polls them, so no stale L2 line may ever shadow the HBM copy.
  SymmetricBuffer(size_t bytes, int device, bool uncached = false);
  bool uncached() const { return uncached_; }
  ~SymmetricBuffer();
  std::string ipc_handle() const;                       // 64 raw bytes
  void open_peers(const std::vector<std::string>& handles, int my_rank);
  void close_peers();
  // Free the local allocation now. Call only after EVERY rank closed its mapping of it
  // (close_peers + barrier): freeing memory a peer still maps makes the next export fail.
  void release();
  uintptr_t local() const { return (uintptr_t)ptr_; }
  uintptr_t peer(int r) const { return (uintptr_t)peers_.at(r); }
  size_t bytes() const { return bytes_; }
  int npeers() const { return (int)peers_.size(); }

 private:
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
  int device_ = 0;
  bool uncached_ = false;
  std::vector<void*> peers_;
  std::vector<bool> opened_;
};

}  // namespace ddlb

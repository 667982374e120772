// C-ABI entry point for one fused scoring launch + pinned host memory helpers.
#include <cstdio>
#include <cstring>
#include <string>

#include "common.h"

namespace ccfd {
int launch_mlp(const ccfd_score_args& a, hipStream_t s);
int launch_mlp_multi(const ccfd_multi_args& m, hipStream_t s);
int launch_lr(const ccfd_score_args& a, hipStream_t s);
int launch_lr_multi(const ccfd_multi_args& m, hipStream_t s);
int launch_gbdt(const ccfd_score_args& a, hipStream_t s);
int launch_gbdt_g32(const ccfd_score_args& a, hipStream_t s);

thread_local std::string g_last_error;
void set_error(const std::string& e) { g_last_error = e; }
}  // namespace ccfd

extern "C" {

const char* ccfd_last_error(void) { return ccfd::g_last_error.c_str(); }

int ccfd_score_launch(const ccfd_score_args* a, void* stream) {
  using namespace ccfd;
  if (a == nullptr || a->blob == nullptr || a->x == nullptr) { set_error("null argument"); return -1; }
  if (a->n < 0) { set_error("n < 0"); return -1; }
  if (a->n == 0) return 0;
  if (a->flags & CCFD_ARG_WIRE_G32) {
    if (a->model != CCFD_MODEL_GBDT) { set_error("G32 rows: GBDT kernel only"); return -3; }
    const bool g20 = (a->flags & CCFD_ARG_WIRE_G20) != 0;     // dword loads: 4-byte aligned rows
    if (reinterpret_cast<uintptr_t>(a->x) & (g20 ? 3 : 15)) {
      set_error(g20 ? "G20 rows must be 4-byte aligned" : "G32 rows must be 16-byte aligned");
      return -3;
    }
    const int rc = launch_gbdt_g32(*a, reinterpret_cast<hipStream_t>(stream));
    if (rc == -2) set_error("G32 launch: bad tree shape (depth 1..8, leaf tables <= 64 KB)");
    else if (rc != 0) set_error(std::string("kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
    return rc;
  }
  if (a->flags & CCFD_ARG_WIRE_W64) {
    if (a->model == CCFD_MODEL_GBDT) { set_error("W64 wire rows: MLP and LR kernels only"); return -3; }
    if (reinterpret_cast<uintptr_t>(a->x) & 15) { set_error("W64 rows must be 16-byte aligned"); return -3; }
  } else if (a->ld < kF || (a->ld & 1) || (reinterpret_cast<uintptr_t>(a->x) & 7)) {
    set_error("x must be 8-byte aligned with an even row stride >= 30");
    return -3;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int rc;
  switch (a->model) {
    case CCFD_MODEL_LR: rc = launch_lr(*a, s); break;
    case CCFD_MODEL_MLP: rc = launch_mlp(*a, s); break;
    case CCFD_MODEL_GBDT: rc = launch_gbdt(*a, s); break;
    default: set_error("unknown model kind"); return -2;
  }
  if (rc != 0) {
    hipError_t e = hipGetLastError();
    set_error(std::string("kernel launch failed: ") + hipGetErrorString(e));
  }
  return rc;
}

int ccfd_score_launch_multi(const ccfd_multi_args* m, void* stream) {
  using namespace ccfd;
  if (m == nullptr || m->base.blob == nullptr || m->base.x == nullptr) { set_error("null argument"); return -1; }
  if (m->base.model != CCFD_MODEL_MLP && m->base.model != CCFD_MODEL_LR) {
    set_error("coalesced launch: MLP and LR models only");
    return -2;
  }
  if (m->nsub < 1 || m->nsub > CCFD_MAX_SUB || m->sub_rows <= 0 ||
      (int64_t)m->base.n > (int64_t)m->nsub * m->sub_rows || (int64_t)m->base.n <= (int64_t)(m->nsub - 1) * m->sub_rows) {
    set_error("coalesced launch: bad nsub / sub_rows / n");
    return -1;
  }
  const bool wire = (m->base.flags & CCFD_ARG_WIRE_W64) != 0;
  if (wire ? (reinterpret_cast<uintptr_t>(m->base.x) & 15) != 0
           : (m->base.ld != kF || (reinterpret_cast<uintptr_t>(m->base.x) & 15) != 0)) {
    set_error("coalesced launch: x must be 16-byte aligned contiguous rows");
    return -3;
  }
  for (int j = 0; j < m->nsub; ++j)
    if (m->sub[j].slot_ctl == nullptr || m->sub[j].done_rec == nullptr) {
      set_error("coalesced launch: every sub-batch needs a completion record");
      return -1;
    }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int rc = m->base.model == CCFD_MODEL_LR ? launch_lr_multi(*m, s) : launch_mlp_multi(*m, s);
  if (rc != 0) set_error(std::string("kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
  return rc;
}

void* ccfd_host_alloc(size_t bytes) {
  void* p = nullptr;
  // NumaUser: pages follow the calling thread's NUMA policy (the rank binds itself to its
  // GPU's socket first, utils/numa.py), so the GPU reads local DRAM over its own PCIe root.
  hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocNumaUser);
  if (e != hipSuccess) {
    ccfd::set_error(std::string("hipHostMalloc: ") + hipGetErrorString(e));
    return nullptr;
  }
  return p;
}

int ccfd_host_free(void* p) { return hipHostFree(p) == hipSuccess ? 0 : -1; }

void* ccfd_host_device_ptr(void* host_ptr) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, host_ptr, 0) != hipSuccess) return nullptr;
  return d;
}

}  // extern "C"

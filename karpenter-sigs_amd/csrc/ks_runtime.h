// ks_runtime.h — internals shared by the C-ABI translation units (ks_capi.cpp: Solve,
// ks_cons.cpp: consolidation): the resident problem, device arena helper and kernel launchers.
#pragma once
#include <atomic>
#include <hip/hip_runtime_api.h>

#include <string>
#include <vector>

#include "../../include/karpenter_amd.h"
#include "ks_host.h"

namespace ks {
hipError_t launch_solve(const KsDev& D, const KsWork* works_dev, int nrep, const Plan& pl, int32_t* qorder,
                        uint64_t* skeys, int32_t* svals, void* stemp, size_t stempBytes, hipStream_t st,
                        hipEvent_t mid, const int32_t* fixed_order = nullptr, hipEvent_t* feas = nullptr,
                        int32_t* run_len = nullptr, uint64_t* run_words = nullptr);
hipError_t launch_sims(const KsDev& D, const KsWork* works_dev, int nsims, const Plan& pl, hipStream_t st);
// The topology simulations' kernel alone, and the feasibility launches launch_sims makes before it (a two-phase
// consolidation plan, ks_cons.cpp run_sims).
hipError_t launch_sims_topo(const KsDev& D, const KsWork* w, int n, const Plan& pl, hipStream_t st);
void launch_feasibility(const KsDev& D, hipStream_t st);
void launch_feasibility_nodes(const KsDev& D, hipStream_t st);
// The first nmw simulations (the long multi-node prefixes) on 4-wave workgroups when the problem allows it
// (sims_mw_supported: resource-only pods, no topology), concurrently with the rest.
bool sims_mw_supported(const KsDev& D, const Plan& pl);
hipError_t launch_sims_split(const KsDev& D, const KsWork* works_dev, int nsims, int nmw, const Plan& pl, hipStream_t st,
                             hipStream_t st2, hipEvent_t fork, hipEvent_t join);
Plan make_plan(const KsDims& d, size_t budget, bool sim = false, int wideKO = 0);
size_t queue_sort_temp_bytes(int n);
hipError_t queue_sort(const KsDev& D, uint64_t* keys, int32_t* vals, void* temp, size_t tempBytes, int32_t* out,
                      hipStream_t st);
hipError_t rank_from_order(const int32_t* order, int32_t* rank, int n, hipStream_t st);
// consolidation record headers + device-side record invariants (ks_queue.hip k_rec_headers)
hipError_t rec_headers(const int32_t* recs, int ns, int recWords, int TW, const int32_t* tplBeg, int ntpl, int32_t* hdr,
                       unsigned long long* status, unsigned* counter, unsigned long long* statusOut, hipStream_t st);
// entry_sim null: one run segment (a Solve's queue); strict: also the pods' template-toleration sets and flags
hipError_t sim_run_lengths(const int32_t* podmap, const int32_t* entry_sim, const int64_t* pod_req, const uint64_t* pod_s0,
                           const int32_t* pod_flags, int R, int n, uint64_t* words, int32_t* run_len, hipStream_t st,
                           bool strict = false);
hipError_t sim_queue_sort(const int32_t* rank, const int32_t* entries, const int32_t* entry_sim, int n, int rbits,
                          int sbits, uint64_t* keys, int32_t* vals, void* temp, size_t tempBytes, int32_t* out,
                          hipStream_t st);

// One hipMalloc carved into 256-byte aligned arrays.
struct Arena {
  size_t total = 0;
  size_t add(size_t bytes) {
    size_t off = total;
    total += (bytes + 255) & ~(size_t)255;
    return off;
  }
};

void set_last_error(const std::string& m);
}  // namespace ks

#define HIPCHK(x)                                                                                         \
  do {                                                                                                    \
    hipError_t e_ = (x);                                                                                  \
    if (e_ != hipSuccess) throw ks::KsError(KS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// The encoded problem resident in HBM (ks_problem_create = NewScheduler).
struct ks_problem {
  std::atomic<int> refs{1};  // the handle + every ks_results that renders from it
  ks::Host host;
  ks::KsDev dev{};
  void* dbuf = nullptr;
  void* fmbuf = nullptr;  // k_feasibility rows (KsDev::st_fm)
  double fmBytes = 0;     // k_feasibility's algorithmic bytes per launch
  void* fnbuf = nullptr;  // k_feasibility_nodes rows (KsDev::st_fn)
  double fnBytes = 0;     // k_feasibility_nodes's algorithmic bytes per launch
  void* wbuf = nullptr;
  size_t wbytes = 0;
  ks::KsWork* works_dev = nullptr;
  int wreps = 0;
  hipStream_t stream = nullptr;
  int device = -1;
  int lastKO = 0;  // claim capacity of the last launch plan
  int wideKO = 0;  // a Solve of this problem outgrew the default plan's NodeClaim capacity (make_plan's level)
  // NewQueue radix-sort workspace
  uint64_t* skeys = nullptr;
  int32_t* svals = nullptr;
  void* stemp = nullptr;
  size_t stempBytes = 0;
  int32_t* hqorder = nullptr;  // [P] NewQueue order from the host (Host::hostQueue), when pods tie
  ~ks_problem() {
    int prev = -1;
    if (device >= 0 && hipGetDevice(&prev) == hipSuccess && prev != device) (void)hipSetDevice(device);
    if (skeys) (void)hipFree(skeys);
    if (svals) (void)hipFree(svals);
    if (stemp) (void)hipFree(stemp);
    if (hqorder) (void)hipFree(hqorder);
    if (dbuf) (void)hipFree(dbuf);
    if (fmbuf) (void)hipFree(fmbuf);
    if (fnbuf) (void)hipFree(fnbuf);
    if (wbuf) (void)hipFree(wbuf);
    if (works_dev) (void)hipFree(works_dev);
    if (stream) (void)hipStreamDestroy(stream);
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  }
};

namespace ks {
// One C-ABI call on a handle: its buffers and stream live on the device it was created on, so that
// device is made current for the call (an opts->device naming another one is an argument error) and
// the caller's current device is restored afterwards.
struct DeviceGuard {
  int prev = -1;
  DeviceGuard(int dev, const ks_solve_opts* opts) {
    if (opts && opts->device >= 0 && opts->device != dev)
      throw KsError(KS_ERR_ARG, "opts->device " + std::to_string(opts->device) + " is not the device the handle was created on (" +
                                    std::to_string(dev) + ")");
    HIPCHK(hipGetDevice(&prev));
    if (prev != dev) HIPCHK(hipSetDevice(dev));
    (void)hipGetLastError();  // clear a sticky error of an unrelated earlier call: the launches check it
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};
}  // namespace ks

// Upload the host tables to one HBM allocation and point pb->dev at them.
void ks_upload(ks_problem* pb);

// Binary snapshots (ks_capi.cpp): a magic, the format version and the sizes of the shared structs.
namespace ks { struct ArOut; struct ArIn; }
void snapshot_header(ks::ArOut& a, const char magic[8]);
void snapshot_check_header(ks::ArIn& a, const char magic[8]);
char* snapshot_bytes(const std::string& s);

#define API_TRY try {
#define API_CATCH                                  \
  }                                                \
  catch (const ks::KsError& e) {                   \
    ks::set_last_error(e.what());                  \
    return e.code;                                 \
  }                                                \
  catch (const std::exception& e) {                \
    ks::set_last_error(e.what());                  \
    return KS_ERR_PARSE;                           \
  }

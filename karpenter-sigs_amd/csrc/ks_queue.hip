// ks_queue.hip — NewQueue (queue.go:37-43) on the GPU: order the pods by byCPUAndMemoryDescending
// (cpu desc, memory desc, creationTimestamp asc, uid asc; queue.go:83-112).
//
// The comparator is a lexicographic order on four int64 components.  The host rejects exact ties
// (which only identical UIDs can produce), so the order is strict and any correct sort reproduces
// Go's unstable sort.Slice.  Implemented as a least-significant-component-first chain of stable
// hipCUB radix sorts over offset-binary keys, each limited to the component's bit width (a constant
// component costs nothing).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "ks_problem.h"

namespace ks {

__global__ void k_qkeys(const int64_t* sortkey, int comp, int64_t minv, const int32_t* perm, uint64_t* keys,
                        int32_t* vals, int n, int first) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int p = first ? i : perm[i];
  keys[i] = (uint64_t)(sortkey[(int64_t)p * 4 + comp] - minv);
  vals[i] = p;
}

__global__ void k_iota(int32_t* v, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = i;
}

size_t queue_sort_temp_bytes(int n) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (const int32_t*)nullptr, (int32_t*)nullptr, n, 0, 64, (hipStream_t)0);
  return bytes;
}

// keys: 2*n u64, vals: 2*n i32, temp: queue_sort_temp_bytes(n).  Result written to `out`.
hipError_t queue_sort(const KsDev& D, uint64_t* keys, int32_t* vals, void* temp, size_t tempBytes,
                      int32_t* out, hipStream_t st) {
  const KsDims& d = D.d;
  const int n = d.P;
  if (n == 0) return hipSuccess;
  const int blocks = (n + 255) / 256;
  const int32_t* cur = nullptr;
  int buf = 0;
  for (int comp = 3; comp >= 0; comp--) {
    const int bits = d.skBits[comp];
    if (bits == 0) continue;
    uint64_t* kin = keys + (size_t)buf * n;
    int32_t* vin = vals + (size_t)buf * n;
    uint64_t* kout = keys + (size_t)(buf ^ 1) * n;
    int32_t* vout = vals + (size_t)(buf ^ 1) * n;
    hipLaunchKernelGGL(k_qkeys, dim3(blocks), dim3(256), 0, st, D.pod_sortkey, comp, d.skMin[comp], cur, kin, vin, n,
                       cur == nullptr ? 1 : 0);
    size_t tb = tempBytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(temp, tb, kin, kout, vin, vout, n, 0, bits, st);
    if (e != hipSuccess) return e;
    cur = vout;
    buf ^= 1;
  }
  if (cur == nullptr) {
    hipLaunchKernelGGL(k_iota, dim3(blocks), dim3(256), 0, st, out, n);
  } else {
    hipError_t e = hipMemcpyAsync(out, cur, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

}  // namespace ks

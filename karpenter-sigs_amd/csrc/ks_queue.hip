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

// Per-simulation NewQueue (queue.go:37-43) for a batch of consolidation simulations.  Each
// simulation's pods are a subset of the cluster problem's pods, and byCPUAndMemoryDescending is a
// strict total order on them, so a simulation's queue is the global queue order restricted to its
// subset: one radix sort of (simulation, global rank) keys orders every simulation at once and the
// stable sort keeps each simulation's entries at its own CSR offsets.
__global__ void k_sim_keys(const int32_t* rank, const int32_t* entries, const int32_t* entry_sim, int rbits,
                           uint64_t* keys, int32_t* vals, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int p = entries[i];
  keys[i] = ((uint64_t)entry_sim[i] << rbits) | (uint64_t)rank[p];
  vals[i] = p;
}

__global__ void k_rank(const int32_t* order, int32_t* rank, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) rank[order[i]] = i;
}

hipError_t rank_from_order(const int32_t* order, int32_t* rank, int n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rank, dim3((n + 255) / 256), dim3(256), 0, st, order, rank, n);
  return hipGetLastError();
}

// keys: 2*n u64, vals: 2*n i32, temp: queue_sort_temp_bytes(n).  Sorted global pod indices -> out.
hipError_t sim_queue_sort(const int32_t* rank, const int32_t* entries, const int32_t* entry_sim, int n, int rbits,
                          int sbits, uint64_t* keys, int32_t* vals, void* temp, size_t tempBytes, int32_t* out,
                          hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sim_keys, dim3((n + 255) / 256), dim3(256), 0, st, rank, entries, entry_sim, rbits, keys, vals, n);
  size_t tb = tempBytes;
  return hipcub::DeviceRadixSort::SortPairs(temp, tb, keys, keys + n, vals, out, n, 0, rbits + sbits, st);
}

// Runs of identical pods in every simulation's NewQueue order (the LEAN simulation fast path places a run in one
// step while no pod has been pushed back, ks_solve.hip): entry i of the sorted CSR starts a run when it is its
// simulation's first entry or its pod differs from the previous entry's in requests, tolerations (the pod's first
// relaxation state) or the provisionable flag.  One bit per entry, 64 per word (one ballot per wave).
// A Solve's queue (entry_sim null, strict): one segment, and the pods' template-toleration sets and state flags
// (pod_s0 words 2, 3) must match too -- the LEAN Solve's claim runs (ks_solve_body.inc).
__global__ __launch_bounds__(256) void k_sim_run_breaks(const int32_t* podmap, const int32_t* entry_sim,
                                                        const int64_t* pod_req, const uint64_t* pod_s0,
                                                        const int32_t* pod_flags, int R, int n, uint64_t* words,
                                                        int strict) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  bool brk = true;
  if (i < n && i > 0 && (!entry_sim || entry_sim[i] == entry_sim[i - 1])) {
    const int p = podmap[i], q = podmap[i - 1];
    bool same = pod_s0[4 * (int64_t)p] == pod_s0[4 * (int64_t)q] && pod_s0[4 * (int64_t)p + 1] == pod_s0[4 * (int64_t)q + 1] &&
                ((pod_flags[p] ^ pod_flags[q]) & PF_PROVISIONABLE) == 0;
    if (strict)
      same = same && pod_s0[4 * (int64_t)p + 2] == pod_s0[4 * (int64_t)q + 2] &&
             pod_s0[4 * (int64_t)p + 3] == pod_s0[4 * (int64_t)q + 3];
    for (int r = 0; r < R; r++) same = same && pod_req[(int64_t)p * R + r] == pod_req[(int64_t)q * R + r];
    brk = !same;
  }
  const uint64_t b = __ballot(brk ? 1 : 0);
  if ((threadIdx.x & 63) == 0 && i < n) words[i >> 6] = b;
}

// Per entry: the entries from it to the next run start (or the end), i.e. the identical pods left in its run.
__global__ __launch_bounds__(256) void k_sim_run_len(const uint64_t* words, int n, int32_t* run_len) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int nw = (n + 63) >> 6;
  int w = (i + 1) >> 6;
  uint64_t m = w < nw ? words[w] & (~0ull << ((i + 1) & 63)) : 0ull;
  while (m == 0 && ++w < nw) m = words[w];
  const int next = m ? (w << 6) + __builtin_ctzll(m) : n;
  run_len[i] = (next < n ? next : n) - i;
}

hipError_t sim_run_lengths(const int32_t* podmap, const int32_t* entry_sim, const int64_t* pod_req, const uint64_t* pod_s0,
                           const int32_t* pod_flags, int R, int n, uint64_t* words, int32_t* run_len, hipStream_t st,
                           bool strict) {
  if (n == 0) return hipSuccess;
  const int blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_sim_run_breaks, dim3(blocks), dim3(256), 0, st, podmap, entry_sim, pod_req, pod_s0, pod_flags, R,
                     n, words, strict ? 1 : 0);
  hipLaunchKernelGGL(k_sim_run_len, dim3(blocks), dim3(256), 0, st, words, n, run_len);
  return hipGetLastError();
}

}  // namespace ks

namespace ks {

// Consolidation record headers (ks_cons.cpp RecView): per simulation the first RF_HDR words of its record,
// compacted for the host (a world-1 pass downloads these instead of every record's option words), and the
// record invariants the host replay would otherwise read every record for (a lost or stale device store
// becomes a loud error, not a wrong decision): computeConsolidation's action against the NodeClaim count
// (consolidation.go:113-194), NewNodeClaims[0]'s options inside its template's list and numbering RF_NOPT,
// filterByPrice's and filterOutSameType's outputs subsets of their inputs with the recorded counts.
// status[0] = min over failing simulations of (sim << 32 | check), status[1] = min of (sim << 32 | kernel
// error) over simulations reporting one; ~0 when none.  The device-side status words and the block counter
// persist between passes (set once at allocation): the last block to finish publishes the status to
// `statusOut` and resets both, so a pass needs no memset.  `hdr` / `statusOut` may be host-mapped pinned
// memory (the pass then needs no copy either): each block stages its headers in LDS and writes them out
// coalesced.
__global__ __launch_bounds__(256) void k_rec_headers(const int32_t* recs, int ns, int recWords, int TW,
                                                     const int32_t* tplBeg, int ntpl, int32_t* hdr,
                                                     unsigned long long* status, unsigned* counter,
                                                     unsigned long long* statusOut) {
  __shared__ int32_t tile[256 * (RF_HDR + 1)];
  __shared__ unsigned last;
  const int s0 = blockIdx.x * blockDim.x, s = s0 + threadIdx.x;
  if (s < ns) {
    const int32_t* r = recs + (size_t)s * recWords;
    int32_t h[RF_HDR];
    for (int i = 0; i < RF_HDR; i++) {
      h[i] = r[i];
      tile[threadIdx.x * (RF_HDR + 1) + i] = h[i];
    }
    int bad = 0;
    if (h[RF_ACTION] < CA_NOOP || h[RF_ACTION] > CA_ERROR) bad = 1;
    else if (h[RF_NCLAIMS] < 0 || h[RF_HOSTINCR] < h[RF_NCLAIMS]) bad = 2;
    else if (h[RF_ACTION] == CA_DELETE && h[RF_NCLAIMS] != 0) bad = 3;
    else if (h[RF_ACTION] == CA_REPLACE && h[RF_NCLAIMS] != 1) bad = 4;
    else if (h[RF_NCLAIMS] > 0) {
      if (h[RF_TPL] < 0 || h[RF_TPL] >= ntpl) {
        bad = 5;
      } else {
        const int nIT = tplBeg[h[RF_TPL] + 1] - tplBeg[h[RF_TPL]];
        const uint32_t* o = (const uint32_t*)r + RF_HDR;
        int nopt = 0, nprice = 0, nsame = 0;
        for (int w = 0; w < TW; w++) {
          const int lo = w * 32;
          const uint32_t valid = nIT >= lo + 32 ? ~0u : nIT > lo ? (1u << (nIT - lo)) - 1u : 0u;
          const uint32_t a = o[w], b = o[TW + w], c = o[2 * TW + w];
          if (a & ~valid) bad = 6;
          if ((b & ~a) || (c & ~b)) bad = bad ? bad : 7;
          nopt += __popc(a);
          nprice += __popc(b);
          nsame += __popc(c);
        }
        if (!bad && (nopt != h[RF_NOPT] || nopt == 0)) bad = 8;
        if (!bad && (nprice != h[RF_NPRICE] || nsame != h[RF_NSAME])) bad = 9;
      }
    }
    if (bad) atomicMin(status, ((unsigned long long)s << 32) | (unsigned)bad);
    if (h[RF_ERROR] != KE_OK) atomicMin(status + 1, ((unsigned long long)s << 32) | (unsigned)h[RF_ERROR]);
  }
  __syncthreads();
  const int nb = ns - s0 < (int)blockDim.x ? ns - s0 : (int)blockDim.x;
  for (int w = threadIdx.x; w < nb * RF_HDR; w += blockDim.x)
    hdr[(size_t)s0 * RF_HDR + w] = tile[(w / RF_HDR) * (RF_HDR + 1) + w % RF_HDR];
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(counter, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (last && threadIdx.x < 2) {  // every block's status atomics are done: publish and reset
    __threadfence();
    statusOut[threadIdx.x] = atomicExch(status + threadIdx.x, ~0ull);
    if (threadIdx.x == 0) atomicExch(counter, 0u);
    __threadfence_system();
  }
}

hipError_t rec_headers(const int32_t* recs, int ns, int recWords, int TW, const int32_t* tplBeg, int ntpl, int32_t* hdr,
                       unsigned long long* status, unsigned* counter, unsigned long long* statusOut, hipStream_t st) {
  if (ns <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_rec_headers, dim3((ns + 255) / 256), dim3(256), 0, st, recs, ns, recWords, TW, tplBeg, ntpl, hdr,
                     status, counter, statusOut);
  return hipGetLastError();
}

}  // namespace ks

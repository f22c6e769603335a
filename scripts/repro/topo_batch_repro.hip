// Standalone reproducer for the batched topology node test (ks_solve.hip topo_node_stateK, DESIGN §3
// "A miscompile of divergent loop exits").  The same loop nest -- groups in chunks of 4, nodes in blocks of
// 4, a per-lane `continue` for unlabelled nodes and a uniform `break` at the chunk's end -- evaluated on
// random inputs, against the one-node-at-a-time form.  Prints the number of disagreeing (lane, node) pairs.
// Build: hipcc -O3 --offload-arch=gfx950 topo_batch_repro.hip -o topo_batch_repro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef REPRO_NOBREAK
#define REPRO_NOBREAK 0
#endif
#ifndef REPRO_SELECT
#define REPRO_SELECT 0
#endif
#ifndef REPRO_TAG
#define REPRO_TAG "default"
#endif
#ifndef REPRO_KN
#define REPRO_KN 4
#endif

constexpr int G = 8, NV = 256, N = 256, TRIALS = 4096;
enum { TG_SPREAD = 0, TG_AFFINITY = 1, TG_ANTI = 2 };

struct In {
  int type[G], skew[G], tmin[G];
  unsigned long long t_mask, t_sel;
};

__device__ __forceinline__ int serial1(const In& x, const int* dom, const int* cnt, const unsigned char* has, int n) {
  int st = 1;
  for (unsigned long long m = x.t_mask; m; m &= m - 1) {
    const int g = __builtin_ctzll(m);
    const int v = dom[g * N + n];
    if (v < 0) {
      st = 2;
      continue;
    }
    const int c = cnt[g * NV + v];
    if (c < 0) return 0;
    const bool self = (x.t_sel >> g) & 1ull;
    if (x.type[g] == TG_SPREAD) {
      if ((long long)c + (int)self - x.tmin[g] > x.skew[g]) return 0;
    } else if (x.type[g] == TG_AFFINITY) {
      if (!has[g * NV + v]) return 0;
      if (x.tmin[g] ? c == 0 : !self) return 0;
    } else if (c != 0 || !has[g * NV + v]) {
      return 0;
    }
  }
  return st;
}

template <int KN>
__device__ __forceinline__ void batched(const In& x, const int* dom, const int* cnt, const unsigned char* has,
                                        const int* c, int* st) {
  constexpr int TGC = 4;
  for (unsigned long long m = x.t_mask; m;) {
    int gs[TGC];
#pragma unroll
    for (int j = 0; j < TGC; j++) {
      gs[j] = m ? __builtin_ctzll(m) : -1;
      m &= m - 1;
    }
    int v[TGC][KN], cn[TGC][KN];
#pragma unroll
    for (int j = 0; j < TGC; j++)
#pragma unroll
      for (int i = 0; i < KN; i++) v[j][i] = gs[j] >= 0 ? dom[gs[j] * N + c[i]] : 0;
#pragma unroll
    for (int j = 0; j < TGC; j++)
#pragma unroll
      for (int i = 0; i < KN; i++) cn[j][i] = (gs[j] >= 0 && v[j][i] >= 0) ? cnt[gs[j] * NV + v[j][i]] : 0;
#pragma unroll
    for (int j = 0; j < TGC; j++) {
#if REPRO_NOBREAK
      if (gs[j] >= 0) {
#else
      if (gs[j] < 0) break;
      {
#endif
      const int g = gs[j], type = x.type[g];
      const bool self = (x.t_sel >> g) & 1ull;
#pragma unroll
      for (int i = 0; i < KN; i++) {
#if REPRO_SELECT
        const int cc = cn[j][i];
        const bool hv = has[g * NV + (v[j][i] < 0 ? 0 : v[j][i])] != 0;
        const bool sp = (long long)cc + (int)self - x.tmin[g] <= x.skew[g];
        const bool af = hv && (x.tmin[g] ? cc != 0 : self);
        const bool an = cc == 0 && hv;
        const bool pass = cc >= 0 && (type == TG_SPREAD ? sp : type == TG_AFFINITY ? af : an);
        const bool unl = v[j][i] < 0;
        st[i] = unl ? (st[i] == 1 ? 2 : st[i]) : (pass ? st[i] : 0);
#else
        if (v[j][i] < 0) {
          if (st[i] == 1) st[i] = 2;
          continue;
        }
        const int cc = cn[j][i];
        bool pass;
        if (cc < 0) pass = false;
        else if (type == TG_SPREAD) pass = (long long)cc + (int)self - x.tmin[g] <= x.skew[g];
        else if (type == TG_AFFINITY) pass = has[g * NV + v[j][i]] && (x.tmin[g] ? cc != 0 : self);
        else pass = cc == 0 && has[g * NV + v[j][i]];
        if (!pass) st[i] = 0;
#endif
      }
      }
    }
  }
}

__global__ __launch_bounds__(64) void k(const In* ins, const int* dom, const int* cnt, const unsigned char* has,
                                        int* bad) {
  const In& x = ins[blockIdx.x];
  int c[4], st[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    c[i] = (threadIdx.x + 64 * i) % N;
    st[i] = ((threadIdx.x * 7 + i * 13 + blockIdx.x) % 5) != 0 ? 1 : 0;  // some nodes already failed
  }
  int s1[4];
#pragma unroll
  for (int i = 0; i < 4; i++) s1[i] = st[i] ? serial1(x, dom, cnt, has, c[i]) : 0;
  batched<REPRO_KN>(x, dom, cnt, has, c, st);
#pragma unroll
  for (int i = 0; i < REPRO_KN; i++)
    if (st[i] != s1[i]) atomicAdd(bad, 1);
}

int main() {
  srand(7);
  std::vector<In> ins(TRIALS);
  for (auto& x : ins) {
    for (int g = 0; g < G; g++) {
      x.type[g] = rand() % 3;
      x.skew[g] = 1 + rand() % 3;
      x.tmin[g] = rand() % 2;
    }
    x.t_mask = (unsigned long long)(rand() & ((1 << G) - 1));
    x.t_sel = (unsigned long long)(rand() & ((1 << G) - 1));
  }
  std::vector<int> dom(G * N), cnt(G * NV);
  std::vector<unsigned char> has(G * NV);
  for (auto& d : dom) d = rand() % 10 == 0 ? -1 : rand() % NV;
  for (auto& c : cnt) c = rand() % 8 == 0 ? -1 : rand() % 4;
  for (auto& h : has) h = rand() % 4 != 0;
  In* dIns;
  int *dDom, *dCnt, *dBad;
  unsigned char* dHas;
  hipMalloc(&dIns, sizeof(In) * TRIALS);
  hipMalloc(&dDom, 4 * dom.size());
  hipMalloc(&dCnt, 4 * cnt.size());
  hipMalloc(&dHas, has.size());
  hipMalloc(&dBad, 4);
  hipMemcpy(dIns, ins.data(), sizeof(In) * TRIALS, hipMemcpyHostToDevice);
  hipMemcpy(dDom, dom.data(), 4 * dom.size(), hipMemcpyHostToDevice);
  hipMemcpy(dCnt, cnt.data(), 4 * cnt.size(), hipMemcpyHostToDevice);
  hipMemcpy(dHas, has.data(), has.size(), hipMemcpyHostToDevice);
  hipMemset(dBad, 0, 4);
  hipLaunchKernelGGL(k, dim3(TRIALS), dim3(64), 0, 0, dIns, dDom, dCnt, dHas, dBad);
  int bad = -1;
  hipMemcpy(&bad, dBad, 4, hipMemcpyDeviceToHost);
  printf("topo_batch_repro[%s]: %d of %d (lane, node) decisions differ between the batched and serial forms\n", REPRO_TAG, bad,
         TRIALS * 64 * 4);
  return 0;
}

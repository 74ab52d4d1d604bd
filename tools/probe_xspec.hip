// probe_xspec.hip -- diagnostic only (not linked into libppfit): the
// headline data pass's launch geometry and byte pattern without the FFT
// (VERDICT r05 next #3), to tell the geometry's memory ceiling apart from
// the FFT's per-row latency.  k_data_xspec<10>: one 4-wave workgroup per
// subint, wave w takes rows w, w + 4, ... of its 64; the row (16 KB) is
// loaded coalesced into registers (lane j: z[j + 64 m]), moved to the wave's
// LDS buffer, the next row's load issued, then per harmonic pair (k, N - k)
// the template row M (L2-resident) is read and X = Z conj(M) written (16.6 KB
// per row, 1040 cells).  Modes: 0 no barrier; 1 the two per-group block
// barriers of the guess accumulation; 2 = 0 at three workgroups per CU (half
// the LDS buffer, the row moved in two halves).
#include <hip/hip_runtime.h>
#include "ppfit_device.hpp"

using namespace ppf;

namespace {
constexpr int N = 1024, NHP = 1040, NCH = 64;

template <int MODE>
__device__ __forceinline__ void body(const double* __restrict__ data, const double2* __restrict__ M,
                                     double2* __restrict__ X, double2* buf) {
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const double* drow0 = data + (size_t)c * NCH * 2 * N;
  WaveRow<10> row;
  row.load(drow0 + (size_t)w * 2 * N, lane);
  for (int g = 0; g < NCH / 4; ++g) {
    const int n = 4 * g + w;
    const double2* Mr = M + (size_t)n * NHP;
    // row -> LDS (MODE 2: the first half only, the buffer is half size)
    constexpr int LI = 16;
#pragma unroll
    for (int i = 0; i < LI; ++i) {
      const int j = lane + 64 * i;
      if (MODE != 2 || i < LI / 2) buf[j] = cmk(row.x[i], row.y[i]);
    }
    if (n + 4 < NCH) row.load(drow0 + (size_t)(n + 4) * 2 * N, lane);
    double2* Xr = X + ((size_t)c * NCH + n) * NHP;
#pragma unroll 2
    for (int i = 0; i < 9; ++i) {
      const int k = min(lane + 64 * i, N / 2);
      const int kb = MODE == 2 ? (k & (N / 2 - 1)) : k;
      const int kn = MODE == 2 ? ((N - k) & (N / 2 - 1)) : ((N - k) & (N - 1));
      const double2 zk = buf[kb], zn = buf[kn];
      const double2 mk = Mr[k], mn = Mr[N - k];
      if (lane + 64 * i <= N / 2) {
        st_stream(cmulc(zk, mk), Xr + k);
        if (k < N / 2) st_stream(cmulc(zn, mn), Xr + N - k);
      }
    }
    for (int k = N + 1 + lane; k < NHP; k += 64) Xr[k] = cmk(0.0, 0.0);
    if (MODE == 1) {
      __syncthreads();
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(256, 2) void k_probe0(const double* d, const double2* M, double2* X) {
  __shared__ double2 bufs[4][kFft1024Slots];
  __shared__ double2 pad[416];  // k_data_xspec's twiddle table and metadata
  if (threadIdx.x == 0) pad[0] = cmk(0.0, 0.0);
  body<0>(d, M, X, bufs[threadIdx.x >> 6]);
}
__global__ __launch_bounds__(256, 2) void k_probe1(const double* d, const double2* M, double2* X) {
  __shared__ double2 bufs[4][kFft1024Slots];
  __shared__ double2 pad[416];
  if (threadIdx.x == 0) pad[0] = cmk(0.0, 0.0);
  body<1>(d, M, X, bufs[threadIdx.x >> 6]);
}
__global__ __launch_bounds__(256, 3) void k_probe2(const double* d, const double2* M, double2* X) {
  __shared__ double2 bufs[4][kFft1024Slots / 2];
  body<2>(d, M, X, bufs[threadIdx.x >> 6]);
}
}  // namespace

extern "C" int probe_xspec(int mode, int nsub, const double* d, const double2* M, double2* X,
                           void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (mode == 0) hipLaunchKernelGGL(k_probe0, dim3(nsub), dim3(256), 0, st, d, M, X);
  else if (mode == 1) hipLaunchKernelGGL(k_probe1, dim3(nsub), dim3(256), 0, st, d, M, X);
  else hipLaunchKernelGGL(k_probe2, dim3(nsub), dim3(256), 0, st, d, M, X);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

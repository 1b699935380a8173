// Losses of the training step (row a6): nn.BCELoss on the sigmoid head (1 class) and
// nn.CrossEntropyLoss on the logits (n classes) — PMU/trainer/unet_trainer.py:23,30-37 — and the
// Probabilistic U-Net's summed CrossEntropyLoss (probabilistic_unet.py:286-304).
//
// Forward: one streaming pass, each thread accumulating its grid-stride elements in fp64, a fixed-
// order block tree, per-block partials, then one block summing the partials in index order:
// deterministic, no atomics.  Backward: one elementwise pass from (input, target, upstream grad) —
// the torch formulas (BCE: (y - t) / max(y (1 - y), 1e-12); CE: softmax - onehot), scaled on the
// device by the upstream gradient and 1/n (mean), so nothing syncs with the host.
// HBM-bound: c2 reads 2 x 8.4 MB (y, t) per pass.
#include "pmu_common.h"

namespace {

constexpr int LT = 256;        // threads per block
constexpr int LMAXB = 1024;    // partial-sum blocks

int loss_blocks(long long n) {
  long long g = (n + LT * 8 - 1) / (LT * 8);
  if (g < 1) g = 1;
  if (g > LMAXB) g = LMAXB;
  return (int)g;
}

// block sum of two doubles in fixed order; thread 0 writes part[blockIdx.x][0..1]
__device__ void block_sum2(double a, double b, double* part) {
  __shared__ double ra[LT], rb[LT];
  ra[threadIdx.x] = a;
  rb[threadIdx.x] = b;
  __syncthreads();
  for (int o = LT / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      ra[threadIdx.x] += ra[threadIdx.x + o];
      rb[threadIdx.x] += rb[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = ra[0];
    part[2 * blockIdx.x + 1] = rb[0];
  }
}

__device__ __forceinline__ float bce_elem(float y, float t) {
  // torch binary_cross_entropy: log terms clamped at -100
  const float ly = fmaxf(logf(y), -100.f), l1y = fmaxf(logf(1.f - y), -100.f);
  return -(t * ly + (1.f - t) * l1y);
}

__global__ __launch_bounds__(LT) void bce_fwd_kernel(const float* __restrict__ y, const float* __restrict__ t,
                                                     long long n, float* __restrict__ each, double* __restrict__ part) {
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * LT + threadIdx.x; i < n; i += (long long)gridDim.x * LT) {
    const float l = bce_elem(y[i], t[i]);
    if (each) each[i] = l;
    s += (double)l;
  }
  if (part) block_sum2(s, 0.0, part);
}

// loss[0] = sum(part[:,0]) * (mean ? 1/denom : 1), denom = count (part[:,1]) or n
__global__ __launch_bounds__(LT) void loss_final_kernel(const double* __restrict__ part, int G, int reduction,
                                                        long long n, int use_count, float* __restrict__ loss,
                                                        float* __restrict__ count_out) {
  double s = 0.0, c = 0.0;
  for (int g = threadIdx.x; g < G; g += LT) {
    s += part[2 * g];
    c += part[2 * g + 1];
  }
  __shared__ double ra[LT], rb[LT];
  ra[threadIdx.x] = s;
  rb[threadIdx.x] = c;
  __syncthreads();
  for (int o = LT / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      ra[threadIdx.x] += ra[threadIdx.x + o];
      rb[threadIdx.x] += rb[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double denom = use_count ? rb[0] : (double)n;
    loss[0] = (float)(reduction == 1 ? ra[0] / denom : ra[0]);
    if (count_out) count_out[0] = (float)denom;
  }
}

// dy = g * (y - t) / max(y (1 - y), 1e-12), g = gout[0] (/ n for mean) or gout[i] (none)
__global__ __launch_bounds__(LT) void bce_bwd_kernel(const float* __restrict__ y, const float* __restrict__ t,
                                                     long long n, int reduction, const float* __restrict__ gout,
                                                     float* __restrict__ dy) {
  const float gs = reduction == 0 ? 0.f : gout[0] * (reduction == 1 ? (float)(1.0 / (double)n) : 1.f);
  for (long long i = (long long)blockIdx.x * LT + threadIdx.x; i < n; i += (long long)gridDim.x * LT) {
    const float yv = y[i];
    const float g = reduction == 0 ? gout[i] : gs;
    dy[i] = g * (yv - t[i]) / fmaxf((1.f - yv) * yv, 1e-12f);
  }
}

// cross entropy per pixel of logits x[n][k][p] (NCHW): lse - x[target]; ignore_index pixels: 0
__global__ __launch_bounds__(LT) void ce_fwd_kernel(const float* __restrict__ x, const long long* __restrict__ tgt,
                                                    int N, int K, long long HW, long long ignore,
                                                    float* __restrict__ each, double* __restrict__ part) {
  double s = 0.0, c = 0.0;
  const long long P = (long long)N * HW;
  for (long long i = (long long)blockIdx.x * LT + threadIdx.x; i < P; i += (long long)gridDim.x * LT) {
    const long long n = i / HW, p = i - n * HW;
    const float* xp = x + n * K * HW + p;
    const long long tv = tgt[i];
    float l = 0.f;
    if (tv != ignore) {
      float m = -INFINITY;
      for (int k = 0; k < K; ++k) m = fmaxf(m, xp[k * HW]);
      float se = 0.f;
      for (int k = 0; k < K; ++k) se += expf(xp[k * HW] - m);
      // a target outside [0, K) that is not ignore_index: torch raises; no host sync here, so the
      // pixel's loss (and the reduced loss) is NaN and the debug build records the index
      const bool tok = tv >= 0 && tv < K;
      PMU_DCHECK(tok, PMU_DBG_INDEX);
      l = tok ? (m + logf(se)) - xp[(long long)tv * HW] : __builtin_nanf("");
      c += 1.0;
    }
    if (each) each[i] = l;
    s += (double)l;
  }
  if (part) block_sum2(s, c, part);
}

// dx[n][k][p] = g * (softmax_k - [k == t]); g = gout[0] / count (mean), gout[0] (sum), gout[i] (none)
__global__ __launch_bounds__(LT) void ce_bwd_kernel(const float* __restrict__ x, const long long* __restrict__ tgt,
                                                    int N, int K, long long HW, long long ignore, int reduction,
                                                    const float* __restrict__ gout, const float* __restrict__ count,
                                                    float* __restrict__ dx) {
  const float gs = reduction == 0 ? 0.f : (reduction == 1 ? gout[0] / count[0] : gout[0]);
  const long long P = (long long)N * HW;
  for (long long i = (long long)blockIdx.x * LT + threadIdx.x; i < P; i += (long long)gridDim.x * LT) {
    const long long n = i / HW, p = i - n * HW;
    const float* xp = x + n * K * HW + p;
    float* dp = dx + n * K * HW + p;
    const long long tv = tgt[i];
    if (tv == ignore) {
      for (int k = 0; k < K; ++k) dp[k * HW] = 0.f;
      continue;
    }
    if (tv < 0 || tv >= K) {  // out-of-range target (see ce_fwd_kernel): NaN gradient
      for (int k = 0; k < K; ++k) dp[k * HW] = __builtin_nanf("");
      continue;
    }
    const float g = reduction == 0 ? gout[i] : gs;
    float m = -INFINITY;
    for (int k = 0; k < K; ++k) m = fmaxf(m, xp[k * HW]);
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += expf(xp[k * HW] - m);
    const float inv = 1.f / se;
    for (int k = 0; k < K; ++k) {
      const float sm = expf(xp[k * HW] - m) * inv;
      dp[k * HW] = g * (sm - (k == (int)tv ? 1.f : 0.f));
    }
  }
}

}  // namespace

extern "C" size_t pmu_loss_ws(long long n) { return (size_t)loss_blocks(n) * 2 * sizeof(double); }

extern "C" int pmu_bce_fwd(const float* y, const float* t, long long n, int reduction, float* loss, double* ws,
                           float* count_out, void* stream) {
  PMU_REQUIRE(y && t && loss && n > 0 && reduction >= 0 && reduction <= 2 && (reduction == 0 || ws));
  const int G = loss_blocks(n);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bce_fwd_kernel, dim3(G), dim3(LT), 0, st, y, t, n, reduction == 0 ? loss : nullptr,
                     reduction == 0 ? nullptr : ws);
  PMU_CHECK_LAUNCH();
  if (reduction != 0) {
    hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(LT), 0, st, (const double*)ws, G, reduction, n, 0, loss,
                       count_out);
    PMU_CHECK_LAUNCH();
  }
  return PMU_OK;
}

extern "C" int pmu_bce_bwd(const float* y, const float* t, long long n, int reduction, const float* gout, float* dy,
                           void* stream) {
  PMU_REQUIRE(y && t && gout && dy && n > 0 && reduction >= 0 && reduction <= 2);
  hipLaunchKernelGGL(bce_bwd_kernel, dim3(loss_blocks(n) * 4), dim3(LT), 0, (hipStream_t)stream, y, t, n, reduction,
                     gout, dy);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_ce_fwd(const float* x, const long long* tgt, int N, int K, long long HW, int reduction,
                          long long ignore_index, float* loss, double* ws, float* count_out, void* stream) {
  PMU_REQUIRE(x && tgt && loss && N > 0 && K > 0 && HW > 0 && reduction >= 0 && reduction <= 2);
  PMU_REQUIRE(reduction == 0 || ws);
  const long long P = (long long)N * HW;
  const int G = loss_blocks(P);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(G), dim3(LT), 0, st, x, tgt, N, K, HW, ignore_index,
                     reduction == 0 ? loss : nullptr, reduction == 0 ? nullptr : ws);
  PMU_CHECK_LAUNCH();
  if (reduction != 0) {
    hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(LT), 0, st, (const double*)ws, G, reduction, P, 1, loss,
                       count_out);
    PMU_CHECK_LAUNCH();
  }
  return PMU_OK;
}

extern "C" int pmu_ce_bwd(const float* x, const long long* tgt, int N, int K, long long HW, int reduction,
                          long long ignore_index, const float* gout, const float* count, float* dx, void* stream) {
  PMU_REQUIRE(x && tgt && gout && dx && N > 0 && K > 0 && HW > 0 && reduction >= 0 && reduction <= 2);
  PMU_REQUIRE(reduction != 1 || count);
  hipLaunchKernelGGL(ce_bwd_kernel, dim3(loss_blocks((long long)N * HW) * 4), dim3(LT), 0, (hipStream_t)stream, x, tgt,
                     N, K, HW, ignore_index, reduction, gout, count, dx);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

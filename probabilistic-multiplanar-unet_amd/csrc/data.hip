// Data-side kernels on gfx950: generic Dice sums, the multi-planar slicer and 3-view volume fusion.
//
// Slicer (PMU/utils/mri_dataset.py:11-143).  A scan is uploaded once (f64, as nibabel's get_fdata
// returns it) and re-laid out per view so that every slice of every view is one contiguous
// p_a x p_b block:   view 0: [i][j][k]   view 1: [j][i][k]   view 2: [k][i][j]
// (pad_dimensions' zero padding at the end of the argmin axis is applied while re-laying out).
// A training batch is then a pure contiguous gather of B slices with the per-slice max
// normalisation of preprocess() fused in (f64 divide, f32 store: bit-identical to the reference's
// numpy f64 arithmetic followed by .float()).  Per-slice maxima (normalisation and the foreground
// filter of the index map) come from one reduction per view.
//
// Fusion (PMU/eval.py:157-203).  Per-view stacked slice predictions -> the three volumes in the
// view-0 frame (eval's permute(2,1,0,3) / permute(2,1,3,0)), their average, argmax label map and
// exact per-class Dice counts for each of the 4 volumes, in one pass over the predictions.
#include "pmu_common.h"

namespace {

constexpr int FUSE_CMAX = 8;

// ---------------- Dice sums: (sum a*b, sum a, sum b) ----------------
__global__ __launch_bounds__(256) void dice_sums_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                        long long n, double* __restrict__ out) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const float x = a[e], y = b[e];
    s0 += (double)(x * y);
    s1 += (double)x;
    s2 += (double)y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o, 64);
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(out + 0, s0);
    atomicAdd(out + 1, s1);
    atomicAdd(out + 2, s2);
  }
}

// ---------------- slicer: per-view layout of a padded scan ----------------
// in: [d0][d1][d2] f64; padded dims p0 >= d0, p1 >= d1, p2 >= d2 (zeros outside).
// view 0 and 1 are row copies (k contiguous); view 2 transposes each (j,k) plane through LDS.
__global__ __launch_bounds__(256) void view_rows_kernel(const double* __restrict__ in, int d0, int d1, int d2, int p0,
                                                        int p1, int p2, int view, double* __restrict__ out) {
  // one block row = one output row of p2 elements: (a, b) = (i, j) for view 0, (j, i) for view 1
  const long long rows = (long long)p0 * p1;
  for (long long r = blockIdx.x; r < rows; r += gridDim.x) {
    int i, j;
    if (view == 0) { i = (int)(r / p1); j = (int)(r % p1); }
    else           { j = (int)(r / p0); i = (int)(r % p0); }
    const bool inside = i < d0 && j < d1;
    const double* src = in + ((long long)i * d1 + j) * d2;
    double* dst = out + r * p2;
    for (int k = threadIdx.x; k < p2; k += blockDim.x) dst[k] = (inside && k < d2) ? src[k] : 0.0;
  }
}

constexpr int TT = 32;
__global__ __launch_bounds__(256) void view2_kernel(const double* __restrict__ in, int d0, int d1, int d2, int p0,
                                                    int p1, int p2, double* __restrict__ out) {
  // out[k][i][j] = in[i][j][k]; block = (32 j) x (32 k) tile of plane i
  __shared__ double t[TT][TT + 1];
  const int i = blockIdx.z;
  const int j0 = blockIdx.y * TT, k0 = blockIdx.x * TT;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 8 rows per pass
  for (int r = ty; r < TT; r += 8) {
    const int j = j0 + r, k = k0 + tx;
    t[r][tx] = (i < d0 && j < d1 && k < d2) ? in[((long long)i * d1 + j) * d2 + k] : 0.0;
  }
  __syncthreads();
  for (int r = ty; r < TT; r += 8) {
    const int k = k0 + r, j = j0 + tx;
    if (k < p2 && j < p1) out[((long long)k * p0 + i) * p1 + j] = t[tx][r];
  }
}

// per-slice max of nslices contiguous slices of px elements each (block per slice)
__global__ __launch_bounds__(256) void slice_max_kernel(const double* __restrict__ v, long long px,
                                                        double* __restrict__ out) {
  __shared__ double red[4];
  const double* s = v + (long long)blockIdx.x * px;
  double m = -INFINITY;
  for (long long e = threadIdx.x; e < px; e += blockDim.x) m = fmax(m, s[e]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// out[b][e] = float(slice[e] / maxv[ids[b]])  (normalize and max != 0), else float(value),
// slice = the f64 slice at device address addr[ids[b]]
__global__ __launch_bounds__(256) void gather_slices_kernel(const long long* __restrict__ addr,
                                                            const double* __restrict__ maxv,
                                                            const int* __restrict__ ids, long long px, int normalize,
                                                            float* __restrict__ out) {
  const int b = blockIdx.y;
  const int id = ids[b];
  PMU_DCHECK(id >= 0 && addr[id] != 0, PMU_DBG_INDEX);
  const double* s = reinterpret_cast<const double*>(addr[id]);
  const double m = maxv ? maxv[id] : 0.0;
  const bool div = normalize && m != 0.0;
  float* d = out + (long long)b * px;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < px; e += (long long)gridDim.x * blockDim.x)
    d[e] = div ? (float)(s[e] / m) : (float)s[e];
}

// ---------------- 3-view fusion ----------------
// v0 [D0][C][D1][D2], v1 [D1][C][D0][D2], v2 [D2][C][D0][D1]: stacked per-slice predictions of
// the three views (probabilities, or logits with softmax applied here when logits != 0).
// truth [D0][D1][D2] labels (float).  counts[v][c][3] += (sum onehot_c*[t==c], sum onehot_c,
// sum [t==c]) for v = view0, view1, view2, average (one-hot of the first maximum).
struct FuseArgs {
  const float *v0, *v1, *v2, *truth;
  int D0, D1, D2, C, logits;
  float* avg;
  int* label;
  double* counts;
};

// register arrays of FUSE_CMAX entries, only the first C live: every loop is unrolled and guarded
__device__ __forceinline__ int argmax_first(const float (&p)[FUSE_CMAX], int C) {
  int am = 0;
  float best = p[0];
#pragma unroll
  for (int c = 1; c < FUSE_CMAX; ++c)
    if (c < C && p[c] > best) { best = p[c]; am = c; }
  return am;
}

__device__ __forceinline__ void softmax_inplace(float (&p)[FUSE_CMAX], int C) {
  float m = p[0];
#pragma unroll
  for (int c = 1; c < FUSE_CMAX; ++c)
    if (c < C) m = fmaxf(m, p[c]);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < FUSE_CMAX; ++c)
    if (c < C) { p[c] = expf(p[c] - m); s += p[c]; }
#pragma unroll
  for (int c = 0; c < FUSE_CMAX; ++c)
    if (c < C) p[c] = p[c] / s;
}

__global__ __launch_bounds__(256) void fuse3view_kernel(FuseArgs a) {
  // block: plane i, row of 32 j, walking every 32-wide k tile; v2 is read [k][j] coalesced in j and
  // transposed in LDS.  The integer counts accumulate in registers over the whole row, are summed
  // over the block in LDS and leave as one exact fp64 atomic per counter per block (per-wave
  // atomics on the same 4*C*3 addresses serialised the kernel).
  __shared__ float t2[FUSE_CMAX][TT][TT + 1];
  __shared__ int red[4][4 * FUSE_CMAX * 2 + FUSE_CMAX];
  const int i = blockIdx.z, j0 = blockIdx.y * TT;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int C = a.C;
  const long long P01 = (long long)a.D0 * a.D1, P02 = (long long)a.D0 * a.D2, P12 = (long long)a.D1 * a.D2;
  int cI[4][FUSE_CMAX], cP[4][FUSE_CMAX], cT[FUSE_CMAX];
#pragma unroll
  for (int c = 0; c < FUSE_CMAX; ++c) {
    cT[c] = 0;
#pragma unroll
    for (int v = 0; v < 4; ++v) { cI[v][c] = 0; cP[v][c] = 0; }
  }
  for (int k0 = 0; k0 < a.D2; k0 += TT) {
    __syncthreads();  // previous tile's t2 reads done
    for (int r = ty; r < TT; r += 8) {
      const int k = k0 + r, j = j0 + tx;
#pragma unroll
      for (int c = 0; c < FUSE_CMAX; ++c)
        if (c < C)
          t2[c][r][tx] = (k < a.D2 && j < a.D1) ? a.v2[((long long)k * C + c) * P01 + (long long)i * a.D1 + j] : 0.f;
    }
    __syncthreads();
    for (int r = ty; r < TT; r += 8) {
      const int j = j0 + r, k = k0 + tx;
      if (j >= a.D1 || k >= a.D2) continue;
      float p0[FUSE_CMAX], p1[FUSE_CMAX], p2[FUSE_CMAX], pa[FUSE_CMAX];
#pragma unroll
      for (int c = 0; c < FUSE_CMAX; ++c) {
        p0[c] = p1[c] = p2[c] = 0.f;
        if (c < C) {
          p0[c] = a.v0[((long long)i * C + c) * P12 + (long long)j * a.D2 + k];
          p1[c] = a.v1[((long long)j * C + c) * P02 + (long long)i * a.D2 + k];
          p2[c] = t2[c][tx][r];
        }
      }
      if (a.logits) {
        softmax_inplace(p0, C);
        softmax_inplace(p1, C);
        softmax_inplace(p2, C);
      }
#pragma unroll
      for (int c = 0; c < FUSE_CMAX; ++c) pa[c] = (p0[c] + p1[c] + p2[c]) / 3.0f;
      const long long vox = ((long long)i * a.D1 + j) * a.D2 + k;
      const int t = (int)a.truth[vox];
      const int m0 = argmax_first(p0, C), m1 = argmax_first(p1, C), m2 = argmax_first(p2, C), ma = argmax_first(pa, C);
#pragma unroll
      for (int c = 0; c < FUSE_CMAX; ++c) {
        if (c >= C) break;
        const int tc = (t == c);
        cT[c] += tc;
        cP[0][c] += (m0 == c); cI[0][c] += (m0 == c) & tc;
        cP[1][c] += (m1 == c); cI[1][c] += (m1 == c) & tc;
        cP[2][c] += (m2 == c); cI[2][c] += (m2 == c) & tc;
        cP[3][c] += (ma == c); cI[3][c] += (ma == c) & tc;
      }
      if (a.avg) {
#pragma unroll
        for (int c = 0; c < FUSE_CMAX; ++c)
          if (c < C) a.avg[((long long)i * C + c) * P12 + (long long)j * a.D2 + k] = pa[c];
      }
      if (a.label) a.label[vox] = ma;
    }
  }
  // wave sums -> LDS -> block sums -> one atomic per counter (exact: integer values in fp64)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < FUSE_CMAX; ++c) {
    if (c >= C) break;
    int v = cT[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wv][8 * FUSE_CMAX + c] = v;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      int x = cI[w][c], y = cP[w][c];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) { x += __shfl_xor(x, o, 64); y += __shfl_xor(y, o, 64); }
      if (lane == 0) {
        red[wv][(w * FUSE_CMAX + c) * 2 + 0] = x;
        red[wv][(w * FUSE_CMAX + c) * 2 + 1] = y;
      }
    }
  }
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid < 4 * C * 3) {
    const int w = tid / (3 * C), rem = tid - w * 3 * C, c = rem / 3, k = rem - c * 3;
    const int slot = (k == 2) ? 8 * FUSE_CMAX + c : (w * FUSE_CMAX + c) * 2 + k;
    const int v = red[0][slot] + red[1][slot] + red[2][slot] + red[3][slot];
    if (v) atomicAdd(a.counts + (w * C + c) * 3 + k, (double)v);
  }
}

}  // namespace

extern "C" int pmu_dice_sums(const float* a, const float* b, long long n, double* out, void* stream) {
  PMU_REQUIRE(a && b && out && n > 0);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(out, 0, 3 * sizeof(double), st) != hipSuccess) return PMU_ERR_ARG;
  long long g = (n + 255) / 256;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(dice_sums_kernel, dim3((unsigned)g), dim3(256), 0, st, a, b, n, out);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_slice_view_layout(const double* vol, int d0, int d1, int d2, int p0, int p1, int p2, int view,
                                     double* out, void* stream) {
  PMU_REQUIRE(vol && out && d0 > 0 && d1 > 0 && d2 > 0 && p0 >= d0 && p1 >= d1 && p2 >= d2 && view >= 0 && view <= 2);
  hipStream_t st = (hipStream_t)stream;
  if (view < 2) {
    const long long rows = (long long)p0 * p1;
    const unsigned g = (unsigned)(rows < 65536 ? rows : 65536);
    hipLaunchKernelGGL(view_rows_kernel, dim3(g), dim3(256), 0, st, vol, d0, d1, d2, p0, p1, p2, view, out);
  } else {
    PMU_REQUIRE(p0 <= 65535);
    hipLaunchKernelGGL(view2_kernel, dim3((unsigned)pmu_cdiv(p2, TT), (unsigned)pmu_cdiv(p1, TT), (unsigned)p0),
                       dim3(256), 0, st, vol, d0, d1, d2, p0, p1, p2, out);
  }
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_slice_max(const double* slices, int nslices, long long px, double* out, void* stream) {
  PMU_REQUIRE(slices && out && nslices > 0 && px > 0);
  hipLaunchKernelGGL(slice_max_kernel, dim3((unsigned)nslices), dim3(256), 0, (hipStream_t)stream, slices, px, out);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_gather_slices(const long long* addr, const double* maxv, const int* ids, int B, long long px,
                                 int normalize, float* out, void* stream) {
  PMU_REQUIRE(addr && ids && out && B > 0 && B <= 65535 && px > 0 && (!normalize || maxv));
  long long gx = (px + 255) / 256;
  if (gx > 64) gx = 64;
  hipLaunchKernelGGL(gather_slices_kernel, dim3((unsigned)gx, (unsigned)B), dim3(256), 0, (hipStream_t)stream, addr,
                     maxv, ids, px, normalize, out);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_fuse3view(const float* v0, const float* v1, const float* v2, const float* truth, int D0, int D1,
                             int D2, int C, int logits, float* avg, int* label, double* counts, void* stream) {
  PMU_REQUIRE(v0 && v1 && v2 && truth && counts && D0 > 0 && D1 > 0 && D2 > 0 && C >= 1 && C <= FUSE_CMAX &&
              D0 <= 65535);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(counts, 0, sizeof(double) * 4 * C * 3, st) != hipSuccess) return PMU_ERR_ARG;
  FuseArgs a{v0, v1, v2, truth, D0, D1, D2, C, logits, avg, label, counts};
  hipLaunchKernelGGL(fuse3view_kernel, dim3(1u, (unsigned)pmu_cdiv(D1, TT), (unsigned)D0), dim3(256), 0, st, a);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

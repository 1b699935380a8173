// ConvTranspose2d(Cin, Cout, kernel 2, stride 2) of Up (PMU/model/unet/unet_parts.py:52)
// forward and backward as GEMMs on f32 MFMA.
//
// The 2x2/s2 transposed conv never overlaps: u[n][2i+a][2j+b][co] = sum_ci x[n][i][j][ci] w[ci][co][a][b] + b[co]
//   forward : C[pix][co*4+ab] = act(x)[pix][ci] . W[ci][co*4+ab]       (M=pixels, N=4Cout, K=Cin)
//   dgrad   : dx[pix][ci] = sum_{ab,co} du[2i+a][2j+b][co] W[ci][co*4+ab] (M=pixels, N=Cin, K=4Cout)
//   wgrad   : dW[ci][co*4+ab] = sum_pix act(x)[pix][ci] du[2i+a][2j+b][co] (M=Cin, N=4Cout, K=pixels, split-K)
// du is the gradient of the concat's "up" half in the skip's frame; the convT output sits at
// (off_h, off_w) inside it (F.pad, unet_parts.py:58-62).
// Tile 128x128x16, 4 waves (2x2), wave tile 64x64 = 2x2 32x32 accumulators, LDS rows k-contiguous.
#include "pmu_common.h"

namespace {

constexpr int GM = 128, GN = 128, GK = 16, GLS = 20;

struct PixDecode {
  int H, W;
  __device__ __forceinline__ void operator()(long long m, int& n, int& i, int& j) const {
    j = (int)(m % W);
    const long long t = m / W;
    i = (int)(t % H);
    n = (int)(t / H);
  }
};

// A[m=pixel][k=channel] = act(frame)
struct ActRowA {
  static constexpr bool KCONTIG = true;
  static constexpr bool VEC = true;
  DevFrame f;
  PixDecode pd;
  __device__ float load(long long m, int k) const {
    int n, i, j; pd(m, n, i, j);
    return frame_value(f, n, i, j, k);
  }
  __device__ float4 load4(long long m, int k) const {
    int n, i, j; pd(m, n, i, j);
    return frame_value4(f, n, i, j, k);
  }
};
// B[k=ci][n] = W[ci*NN + n]
struct WKN_B {
  static constexpr bool KCONTIG = false;
  const float* w;
  int NN;
  __device__ float load(int k, int n) const { return w[(long long)k * NN + n]; }
};
// A[m=pixel][k'=ab*Cout+co] = du gathered
struct DuGatherA {
  static constexpr bool KCONTIG = true;
  static constexpr bool VEC = true;
  const float* du;
  int Hd, Wd, off_h, off_w, Cout;
  PixDecode pd;
  __device__ __forceinline__ long long idx(long long m, int k) const {
    int n, i, j; pd(m, n, i, j);
    const int ab = k / Cout, co = k - ab * Cout;
    const int hh = off_h + 2 * i + (ab >> 1), ww = off_w + 2 * j + (ab & 1);
    return (((long long)n * Hd + hh) * Wd + ww) * Cout + co;
  }
  __device__ float load(long long m, int k) const { return du[idx(m, k)]; }
  __device__ float4 load4(long long m, int k) const {
    if ((Cout & 3) == 0) return *reinterpret_cast<const float4*>(du + idx(m, k));
    return make_float4(du[idx(m, k)], du[idx(m, k + 1)], du[idx(m, k + 2)], du[idx(m, k + 3)]);
  }
};
// B[k'=ab*Cout+co][n=ci] = W[ci][co*4+ab]
struct WT_B {
  static constexpr bool KCONTIG = true;
  const float* w;
  int Cout;
  __device__ float load(int k, int n) const {
    const int ab = k / Cout, co = k - ab * Cout;
    return w[(long long)n * Cout * 4 + co * 4 + ab];
  }
};
// A[m=ci][k=pixel] = act(frame)
struct ActColA {
  static constexpr bool KCONTIG = false;
  static constexpr bool VEC = false;
  DevFrame f;
  PixDecode pd;
  __device__ float load(long long m, long long k) const {
    int n, i, j; pd(k, n, i, j);
    return frame_value(f, n, i, j, (int)m);
  }
  __device__ float4 load4(long long, long long) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
};
// B[k=pixel][n'=ab*Cout+co] = du gathered
struct DuGatherB {
  static constexpr bool KCONTIG = false;
  DuGatherA g;
  __device__ float load(long long k, int n) const { return g.load(k, n); }
};

struct ScatterEp {  // convT forward output
  float* u;
  const float* bias;
  int H, W, Cout;
  PixDecode pd;
  __device__ void store(long long m, int col, float v, int) const {
    int n, i, j; pd(m, n, i, j);
    const int co = col >> 2, a = (col >> 1) & 1, b = col & 1;
    u[(((long long)n * 2 * H + 2 * i + a) * (2 * W) + 2 * j + b) * Cout + co] = v + (bias ? bias[co] : 0.f);
  }
};
struct RowEp {  // plain row-major store C[m][n]
  float* out;
  int ld;
  __device__ void store(long long m, int col, float v, int) const { out[m * ld + col] = v; }
};
struct SlabEp {  // split-K slab ws[split][m][n]
  float* ws;
  int M, N;
  __device__ void store(long long m, int col, float v, int split) const {
    ws[((long long)split * M + m) * N + col] = v;
  }
};

template <class AL, class BL, class EP>
__global__ __launch_bounds__(256, 2) void gemm_kernel(AL al, BL bl, EP ep, long long M, int N, long long K, int cps) {
  __shared__ __attribute__((aligned(16))) float As[GM * GLS];
  __shared__ __attribute__((aligned(16))) float Bs[GN * GLS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const long long m0 = (long long)blockIdx.x * GM;
  const int n0 = blockIdx.y * GN;
  const int split = blockIdx.z;
  const long long nch = (K + GK - 1) / GK;
  const long long c_beg = (long long)split * cps;
  long long c_end = c_beg + cps;
  if (c_end > nch) c_end = nch;
  const int hsel = (lane >> 5) * 8;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  for (long long ch = c_beg; ch < c_end; ++ch) {
    const long long k0 = ch * GK;
    // ---- A tile [GM][GK]
    if constexpr (AL::KCONTIG && AL::VEC) {
      for (int it = tid; it < GM * GK / 4; it += 256) {
        const int ml = it >> 2, kq = (it & 3) * 4;
        const long long m = m0 + ml, k = k0 + kq;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m < M) {
          if (k + 3 < K) v = al.load4(m, (int)k);
          else {
            float t[4];
            for (int e = 0; e < 4; ++e) t[e] = (k + e < K) ? al.load(m, (int)(k + e)) : 0.f;
            v = make_float4(t[0], t[1], t[2], t[3]);
          }
        }
        *reinterpret_cast<float4*>(As + ml * GLS + kq) = v;
      }
    } else if constexpr (AL::KCONTIG) {
      for (int it = tid; it < GM * GK; it += 256) {
        const int ml = it / GK, kl = it % GK;
        const long long m = m0 + ml, k = k0 + kl;
        As[ml * GLS + kl] = (m < M && k < K) ? al.load(m, k) : 0.f;
      }
    } else {
      for (int it = tid; it < GM * GK; it += 256) {
        const int kl = it / GM, ml = it % GM;
        const long long m = m0 + ml, k = k0 + kl;
        As[ml * GLS + kl] = (m < M && k < K) ? al.load(m, k) : 0.f;
      }
    }
    // ---- B tile, stored [GN][GK]
    if constexpr (BL::KCONTIG) {
      for (int it = tid; it < GN * GK; it += 256) {
        const int nl = it / GK, kl = it % GK;
        const int n = n0 + nl;
        const long long k = k0 + kl;
        Bs[nl * GLS + kl] = (n < N && k < K) ? bl.load(k, n) : 0.f;
      }
    } else {
      for (int it = tid; it < GN * GK; it += 256) {
        const int kl = it / GN, nl = it % GN;
        const int n = n0 + nl;
        const long long k = k0 + kl;
        Bs[nl * GLS + kl] = (n < N && k < K) ? bl.load(k, n) : 0.f;
      }
    }
    __syncthreads();
    float av[2][8], bv[2][8];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const float* pa = As + (wm * 64 + f * 32 + (lane & 31)) * GLS + hsel;
      const float4 x0 = *reinterpret_cast<const float4*>(pa), x1 = *reinterpret_cast<const float4*>(pa + 4);
      av[f][0] = x0.x; av[f][1] = x0.y; av[f][2] = x0.z; av[f][3] = x0.w;
      av[f][4] = x1.x; av[f][5] = x1.y; av[f][6] = x1.z; av[f][7] = x1.w;
      const float* pb = Bs + (wn * 64 + f * 32 + (lane & 31)) * GLS + hsel;
      const float4 y0 = *reinterpret_cast<const float4*>(pb), y1 = *reinterpret_cast<const float4*>(pb + 4);
      bv[f][0] = y0.x; bv[f][1] = y0.y; bv[f][2] = y0.z; bv[f][3] = y0.w;
      bv[f][4] = y1.x; bv[f][5] = y1.y; bv[f][6] = y1.z; bv[f][7] = y1.w;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn) acc[fm][fn] = mfma_f32_32x32x2(av[fm][s], bv[fn][s], acc[fm][fn]);
    __syncthreads();
  }
#pragma unroll
  for (int fn = 0; fn < 2; ++fn) {
    const int col = n0 + wn * 64 + fn * 32 + (lane & 31);
    if (col >= N) continue;
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long m = m0 + wm * 64 + fm * 32 + acc_row(r, lane);
        if (m < M) ep.store(m, col, acc[fm][fn][r], split);
      }
  }
}

// dW[ci][co*4+ab] = sum_s ws[s][ci][ab*Cout+co]
__global__ void convT_wreduce_kernel(const float* __restrict__ ws, int nsplit, int Cin, int Cout, float* __restrict__ dw) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // ci*(4Cout) + (ab*Cout+co)
  const long long E = (long long)Cin * 4 * Cout;
  if (e >= E) return;
  float s = 0.f;
  for (int sp = 0; sp < nsplit; ++sp) s += ws[(long long)sp * E + e];
  const int ci = (int)(e / (4 * Cout));
  const int r = (int)(e - (long long)ci * 4 * Cout);
  const int ab = r / Cout, co = r - ab * Cout;
  dw[(long long)ci * 4 * Cout + co * 4 + ab] = s;
}

// per-block partial bias grads over the convT output region of du: part[blk][Cout]
constexpr int CB_PPB = 2048;
__global__ __launch_bounds__(256) void convT_bias_kernel(const float* __restrict__ du, int N, int Hd, int Wd, int off_h,
                                                         int off_w, int Ho, int Wo, int Cout, float* __restrict__ part) {
  __shared__ float red[256];
  const int tid = threadIdx.x;
  const int cpt = Cout < 256 ? Cout : 256;
  const int npg = 256 / cpt;
  const int pg = tid / cpt;
  const long long P = (long long)N * Ho * Wo;
  const long long p0 = (long long)blockIdx.x * CB_PPB;
  for (int c0 = 0; c0 < Cout; c0 += cpt) {
    const int c = c0 + tid % cpt;
    float s = 0.f;
    if (pg < npg && c < Cout) {
      for (int i = pg; i < CB_PPB; i += npg) {
        const long long p = p0 + i;
        if (p >= P) break;
        const int w = (int)(p % Wo);
        const int h = (int)((p / Wo) % Ho);
        const int n = (int)(p / ((long long)Wo * Ho));
        s += du[(((long long)n * Hd + off_h + h) * Wd + off_w + w) * Cout + c];
      }
    }
    red[tid] = s;
    __syncthreads();
    if (pg == 0 && c < Cout) {
      float t = 0.f;
      for (int l = 0; l < npg; ++l) t += red[l * cpt + tid % cpt];
      part[(long long)blockIdx.x * Cout + c] = t;
    }
    __syncthreads();
  }
}

__global__ void rows_sum_f32_kernel(const float* __restrict__ ws, int R, int Wd, float* __restrict__ out) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= Wd) return;
  double s = 0.0;
  for (int r = 0; r < R; ++r) s += ws[(long long)r * Wd + o];
  out[o] = (float)s;
}

static void convT_wgrad_geometry(int N, int H, int W, int Cin, int Cout, int* nsplit, int* cps) {
  const long long K = (long long)N * H * W;
  const long long nch = (K + GK - 1) / GK;
  const int bmn = pmu_cdiv(Cin, GM) * pmu_cdiv(4 * Cout, GN);
  long long s = 1024 / bmn;
  if (s < 1) s = 1;
  if (s > nch) s = nch;
  *cps = (int)((nch + s - 1) / s);
  *nsplit = (int)((nch + *cps - 1) / *cps);
}

}  // namespace

extern "C" int pmu_convT2x2_fwd(const pmu_frame* in, const float* w, const float* bias, int Cout, float* u,
                                void* stream) {
  PMU_REQUIRE(valid_frame(in) && w && u && Cout > 0);
  ActRowA al{make_dev_frame(in), PixDecode{in->H, in->W}};
  const int Cin = al.f.C;
  WKN_B bl{w, 4 * Cout};
  ScatterEp ep{u, bias, in->H, in->W, Cout, PixDecode{in->H, in->W}};
  const long long M = (long long)in->N * in->H * in->W;
  const int N = 4 * Cout;
  const long long nch = (Cin + GK - 1) / GK;
  dim3 grid((unsigned)pmu_cdiv(M, GM), (unsigned)pmu_cdiv(N, GN), 1);
  hipLaunchKernelGGL((gemm_kernel<ActRowA, WKN_B, ScatterEp>), grid, dim3(256), 0, (hipStream_t)stream, al, bl, ep, M,
                     N, (long long)Cin, (int)nch);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_convT2x2_dgrad(const float* du, int Hd, int Wd, int off_h, int off_w, const float* w, int N,
                                  int H, int W, int Cin, int Cout, float* dx, void* stream) {
  PMU_REQUIRE(du && w && dx && N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0);
  PMU_REQUIRE(off_h >= 0 && off_w >= 0 && off_h + 2 * H <= Hd && off_w + 2 * W <= Wd);
  DuGatherA al{du, Hd, Wd, off_h, off_w, Cout, PixDecode{H, W}};
  WT_B bl{w, Cout};
  RowEp ep{dx, Cin};
  const long long M = (long long)N * H * W;
  const long long K = 4LL * Cout;
  dim3 grid((unsigned)pmu_cdiv(M, GM), (unsigned)pmu_cdiv(Cin, GN), 1);
  hipLaunchKernelGGL((gemm_kernel<DuGatherA, WT_B, RowEp>), grid, dim3(256), 0, (hipStream_t)stream, al, bl, ep, M,
                     Cin, K, (int)((K + GK - 1) / GK));
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" size_t pmu_convT2x2_wgrad_ws(int N, int H, int W, int Cin, int Cout) {
  int ns, cps;
  convT_wgrad_geometry(N, H, W, Cin, Cout, &ns, &cps);
  const size_t slab = (size_t)ns * Cin * 4 * Cout * sizeof(float);
  const size_t bias = (size_t)pmu_cdiv((long long)N * 2 * H * 2 * W, CB_PPB) * Cout * sizeof(float);
  return slab > bias ? slab : bias;
}

extern "C" int pmu_convT2x2_wgrad(const float* du, int Hd, int Wd, int off_h, int off_w, const pmu_frame* act,
                                  int Cout, float* dw, float* dbias, float* ws, size_t ws_bytes, void* stream) {
  PMU_REQUIRE(du && valid_frame(act) && dw && ws && Cout > 0);
  const int N = act->N, H = act->H, W = act->W;
  PMU_REQUIRE(off_h >= 0 && off_w >= 0 && off_h + 2 * H <= Hd && off_w + 2 * W <= Wd);
  PMU_REQUIRE(ws_bytes >= pmu_convT2x2_wgrad_ws(N, H, W, act->src[0].C + (act->nsrc > 1 ? act->src[1].C : 0), Cout));
  ActColA al{make_dev_frame(act), PixDecode{H, W}};
  const int Cin = al.f.C;
  DuGatherB bl{DuGatherA{du, Hd, Wd, off_h, off_w, Cout, PixDecode{H, W}}};
  const int NN = 4 * Cout;
  SlabEp ep{ws, Cin, NN};
  int ns, cps;
  convT_wgrad_geometry(N, H, W, Cin, Cout, &ns, &cps);
  const long long K = (long long)N * H * W;
  dim3 grid((unsigned)pmu_cdiv(Cin, GM), (unsigned)pmu_cdiv(NN, GN), (unsigned)ns);
  hipLaunchKernelGGL((gemm_kernel<ActColA, DuGatherB, SlabEp>), grid, dim3(256), 0, (hipStream_t)stream, al, bl, ep,
                     (long long)Cin, NN, K, cps);
  PMU_CHECK_LAUNCH();
  const long long E = (long long)Cin * NN;
  hipLaunchKernelGGL(convT_wreduce_kernel, dim3((unsigned)pmu_cdiv(E, 256)), dim3(256), 0, (hipStream_t)stream,
                     (const float*)ws, ns, Cin, Cout, dw);
  PMU_CHECK_LAUNCH();
  if (dbias) {
    // the slab is consumed; reuse the workspace for the bias partials (same stream => ordered)
    const int R = pmu_cdiv((long long)N * 2 * H * 2 * W, CB_PPB);
    hipLaunchKernelGGL(convT_bias_kernel, dim3((unsigned)R), dim3(256), 0, (hipStream_t)stream, du, N, Hd, Wd, off_h,
                       off_w, 2 * H, 2 * W, Cout, ws);
    PMU_CHECK_LAUNCH();
    hipLaunchKernelGGL(rows_sum_f32_kernel, dim3((unsigned)pmu_cdiv(Cout, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)ws, R, Cout, dbias);
    PMU_CHECK_LAUNCH();
  }
  return PMU_OK;
}

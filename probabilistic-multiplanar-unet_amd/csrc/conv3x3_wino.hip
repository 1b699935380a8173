// 3x3 / pad 1 convolution in fp32 by Winograd F(2x2, 3x3) on f32 MFMA (the forward of nn.Conv2d at
// PMU/model/unet/unet_parts.py:15,18 and its input gradient), the c2 headline path.
//
// Every 2x2 block of output pixels ("Winograd tile") is computed from the 4x4 operand patch d around
// it as  Y = A^T [ (G g G^T) .* (B^T d B) ] A : 16 element-wise products per input/output channel
// pair instead of 36, i.e. the reduction over input channels becomes 16 independent GEMMs
// ("components") of  M[comp][tile][co] = sum_ci V[comp][tile][ci] * U[comp][ci][co].
// All arithmetic is fp32 (transforms with coefficients 0, +-1, +-1/2); the result differs from the
// direct sum only by fp32 rounding (~1e-6 relative), far inside the 1e-3 parity bound.
//
// Block: 512 threads, 64 tiles (8 x 8 -> a 16 x 16 output patch) x 32 output channels.  Wave w owns
// 16 tiles (tile group w & 3) x 16 output channels (half w >> 2) for all 16 components: acc[16] of
// v_mfma_f32_16x16x4_f32 (64 accumulator registers), so the output transform of each (tile, channel)
// is local to its lane, and two waves share each SIMD.  Per chunk of 16 input channels:
//   * the 18 x 18 x 16 operand halo is staged into LDS through the shared frame staging (BN+ReLU,
//     max-pool, F.pad + concat, or BN+ReLU backward applied on the fly, pmu_stage.h);
//   * U (pre-transformed weights, 16 comps x 16 ch x 32 co) is copied into LDS;
//   * per 4-channel MFMA step each lane reads its tile's 4 x 4 patch for one channel (ds_read_b64 of
//     two channels serve two steps; conflict-free through the padded row pitch), forms the 16
//     components of B^T d B in registers and issues 16 MFMAs with U fragments read as ds_read_b128
//     (4 components per read).
// Epilogue: A^T M A per lane (+bias), BN partial sums per block (fwd), or the split dx store (dgrad).
#include <string.h>
#include <stdlib.h>
#include "pmu_stage.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TX = 8, TY = 8;             // Winograd tiles per block
constexpr int OW = 2 * TX, OH = 2 * TY;   // 16 x 16 output pixels
constexpr int HW = OW + 2, HH = OH + 2;   // 18 x 18 halo
constexpr int BK = 16;                    // input channels per chunk
constexpr int LS = BK + 4;                // LDS floats per halo pixel
constexpr int ROWP = HW * LS + 2;         // halo row pitch: tile-row step 2*ROWP = 20 (mod 64) -> b64 patch reads conflict-free
constexpr int A_FLOATS = HH * ROWP;
constexpr int CO = 32;                    // output channels per block
constexpr int U_FLOATS = BK * 16 * CO;    // one chunk of transformed weights
constexpr int NT = 512;                   // 8 waves: 4 tile groups x 2 channel halves
constexpr int NI = 3;                     // halo items per thread: ceil(324 * 4 / 512)

struct WinoArgs {
  DevFrame in;
  const float* wp;    // packed U [co block][chunk][ch 16][comp group 4][co 32][comp 4]
  const float* bias;
  float* out0;
  float* out1;
  float* part;        // [spatial tiles][2][NOUT] BN partial sums (fwd) or null
  float* tee;         // [N][H][W][KC] copy of the staged operand or null
  int NOUT, KC, split, tiles_w, tiles_h, nco;
  int prio;           // 1: waves 4-7 run at s_setprio 1 (PMU_WINO_PRIO, raw kernel)
  int cpb;            // output-channel blocks per workgroup, walked in passes (raw kernel; else 1)
};

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// U = G g G^T for F(2x2, 3x3), G = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1]; one thread per
// (co block, chunk, channel, co) writes its 16 components as 4 float4 (component groups)
__global__ void pack_wino_kernel(const float* __restrict__ w, int Cout, int Cin, int dgrad, float* __restrict__ wp) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  const int nch = (KC + BK - 1) / BK, ncob = (NOUT + CO - 1) / CO;
  const long long total = (long long)ncob * nch * BK * CO;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int col = (int)(e % CO);
    long long r = e / CO;
    const int kl = (int)(r % BK); r /= BK;
    const int ch = (int)(r % nch);
    const int jb = (int)(r / nch);
    const int j = jb * CO + col, k = ch * BK + kl;
    float g[3][3];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        float v = 0.f;
        if (j < NOUT && k < KC)  // dgrad: the input gradient convolves dz with w[co][ci] rotated by 180 degrees
          v = dgrad ? w[((long long)k * Cin + j) * 9 + (2 - a) * 3 + (2 - b)] : w[((long long)j * Cin + k) * 9 + a * 3 + b];
        g[a][b] = v;
      }
    float t[4][3];  // G g
    for (int b = 0; b < 3; ++b) {
      t[0][b] = g[0][b];
      t[1][b] = 0.5f * (g[0][b] + g[1][b] + g[2][b]);
      t[2][b] = 0.5f * (g[0][b] - g[1][b] + g[2][b]);
      t[3][b] = g[2][b];
    }
    float u[16];  // (G g) G^T
    for (int a = 0; a < 4; ++a) {
      u[4 * a + 0] = t[a][0];
      u[4 * a + 1] = 0.5f * (t[a][0] + t[a][1] + t[a][2]);
      u[4 * a + 2] = 0.5f * (t[a][0] - t[a][1] + t[a][2]);
      u[4 * a + 3] = t[a][2];
    }
    float* dst = wp + ((long long)jb * nch + ch) * U_FLOATS;
    for (int gq = 0; gq < 4; ++gq)
      *reinterpret_cast<float4*>(dst + ((kl * 4 + gq) * CO + col) * 4) =
          make_float4(u[4 * gq], u[4 * gq + 1], u[4 * gq + 2], u[4 * gq + 3]);
  }
}

// V = B^T d B, B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]; v[4i + k]
__device__ __forceinline__ void input_transform(const float (&d)[4][4], float (&v)[16]) {
  float t[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t[0][j] = d[0][j] - d[2][j];
    t[1][j] = d[1][j] + d[2][j];
    t[2][j] = d[2][j] - d[1][j];
    t[3][j] = d[1][j] - d[3][j];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[4 * i + 0] = t[i][0] - t[i][2];
    v[4 * i + 1] = t[i][1] + t[i][2];
    v[4 * i + 2] = t[i][2] - t[i][1];
    v[4 * i + 3] = t[i][1] - t[i][3];
  }
}

// One chunk (16 channels) of MFMAs: per 4-channel step each lane reads its tile's 4x4 patch for one
// channel, transforms it, and issues 16 components x 2 channel halves of 16x16x4 MFMAs.  The next
// step's patch and U fragments are loaded before this step's MFMAs (sched_barrier keeps the order).
// MFMA k-slot -> channel: in step ks a lane of k-group kk (= lane >> 4) multiplies channel
// 8*(ks>>1) + 2*kk + (ks&1), so one ds_read_b64 per patch element serves two steps.
__device__ __forceinline__ int wino_chan(int ks, int kk) { return 8 * (ks >> 1) + 2 * kk + (ks & 1); }

// LDS reads of the MFMA loop as explicit instructions: the patch reads must stay single ds_read_b64
// (256 B/clk, conflict-free here; the compiler merges pairs into ds_read2_b64, which banks on 16-lane
// groups mod 32 where the tiles' even pixel steps collide 2-way).  Being asm, the compiler inserts
// no waits for them: wino_chunk waits (lgkmcnt(0)) at the top of each step, before issuing the next
// step's reads, when the reads for this step — issued a whole step of MFMAs earlier — have landed.
template <int OFF>
__device__ __forceinline__ float2 lds_b64(unsigned addr) {
  float2 v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ float4 lds_b128(unsigned addr) {
  float4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)(p);
}

// the 4x4 patch of this lane's tile for a pair of steps (two adjacent channels per element);
// addr = byte address of the patch origin for the pair
__device__ __forceinline__ void wino_load_patch(unsigned addr, float2 (&d)[16]) {
#define PMU_P(I, J) d[4 * I + J] = lds_b64<((I) * ROWP + (J) * LS) * 4>(addr);
  PMU_P(0, 0) PMU_P(0, 1) PMU_P(0, 2) PMU_P(0, 3) PMU_P(1, 0) PMU_P(1, 1) PMU_P(1, 2) PMU_P(1, 3)
  PMU_P(2, 0) PMU_P(2, 1) PMU_P(2, 2) PMU_P(2, 3) PMU_P(3, 0) PMU_P(3, 1) PMU_P(3, 2) PMU_P(3, 3)
#undef PMU_P
}
// U fragments of one step: 16 components (4 x b128); addr = byte address for this lane's channel
__device__ __forceinline__ void wino_load_u(unsigned addr, float4 (&u)[4]) {
  u[0] = lds_b128<0>(addr);
  u[1] = lds_b128<CO * 16>(addr);
  u[2] = lds_b128<2 * CO * 16>(addr);
  u[3] = lds_b128<3 * CO * 16>(addr);
}

template <bool NOXF = false>
__device__ __forceinline__ void wino_mfmas(const float2 (&dp)[16], bool hi, const float4 (&u)[4], f32x4 (&acc)[16]) {
  float dd[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) dd[i][j] = hi ? dp[4 * i + j].y : dp[4 * i + j].x;
  float v[16];
  if (NOXF) {  // timing experiment only (PMU_WINO_EXP=3): no input transform
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = dd[c >> 2][c & 3];
  } else {
    input_transform(dd, v);
  }
  __builtin_amdgcn_sched_barrier(0);  // all 16 components first: the MFMAs then issue back to back
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    acc[4 * g + 0] = mfma16(v[4 * g + 0], u[g].x, acc[4 * g + 0]);
    acc[4 * g + 1] = mfma16(v[4 * g + 1], u[g].y, acc[4 * g + 1]);
    acc[4 * g + 2] = mfma16(v[4 * g + 2], u[g].z, acc[4 * g + 2]);
    acc[4 * g + 3] = mfma16(v[4 * g + 3], u[g].w, acc[4 * g + 3]);
  }
}

// One chunk (16 channels, 4 steps of 16 MFMAs per wave); the next step's operands are read before
// this step's MFMAs (sched_barrier keeps the order).
template <bool NOXF = false>
__device__ __forceinline__ void wino_chunk(const float* As, const float* Us, int pbase, int ubase, int kk,
                                           f32x4 (&acc)[16]) {
  const unsigned pa = lds_addr(As + pbase), ua = lds_addr(Us + ubase) + (unsigned)(2 * kk * 4 * CO * 4 * 4);
  float2 dp[2][16];
  float4 u[2][4];
  wino_load_patch(pa, dp[0]);
  wino_load_u(ua, u[0]);
#pragma unroll
  for (int ks = 0; ks < BK / 4; ++ks) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (ks + 1 < BK / 4) {
      const int n1 = ks + 1;
      if ((n1 & 1) == 0) wino_load_patch(pa + 32 * (n1 >> 1), dp[(n1 >> 1) & 1]);
      // channel 8*(n1>>1) + 2*kk + (n1&1): the kk part is in ua
      wino_load_u(ua + (unsigned)((8 * (n1 >> 1) + (n1 & 1)) * 4 * CO * 4 * 4), u[n1 & 1]);
    }
    __builtin_amdgcn_sched_barrier(0);
    wino_mfmas<NOXF>(dp[(ks >> 1) & 1], ks & 1, u[ks & 1], acc);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// the operand for the weight gradient: the chunk's interior 16 x 16 pixels x 16 channels
__device__ __forceinline__ void wino_tee(const WinoArgs& a, const float* As, int k0, int n, int h0, int w0, int tid) {
  const DevFrame& F = a.in;
#pragma unroll
  for (int i = 0; i < 1024 / NT; ++i) {
    const int u = tid + NT * i;
    const int q = u >> 2, qq = u & 3;
    const int r = q >> 4, c = q & 15;
    const int h = h0 + r, w = w0 + c, kc = k0 + 4 * qq;
    if (h < F.H && w < F.W && kc < a.KC)
      *reinterpret_cast<float4*>(a.tee + (((long long)n * F.H + h) * F.W + w) * a.KC + kc) =
          *reinterpret_cast<const float4*>(As + (r + 1) * ROWP + (c + 1) * LS + 4 * qq);
  }
}

// block geometry shared by both kernels
struct WinoGeo {
  int cob_blk, spatial, n, h0, w0, j0, tg, hh, kk, pbase, ubase;
};
__device__ __forceinline__ WinoGeo wino_geo(const WinoArgs& a) {
  WinoGeo g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware order: the hardware deals consecutive workgroups round-robin over the 8 XCDs; remap
  // so each XCD runs a contiguous range of logical blocks, i.e. the output-channel blocks of one
  // spatial tile share their operand halo through that XCD's L2
  const int nb = gridDim.x, x = blockIdx.x & 7, q = nb >> 3, r = nb & 7;
  const int lb = x * q + (x < r ? x : r) + (blockIdx.x >> 3);
  const int ncog = (a.nco + a.cpb - 1) / a.cpb;  // co-block groups (cpb co-blocks each)
  g.cob_blk = (lb % ncog) * a.cpb;
  int sp = lb / ncog;
  g.spatial = sp;
  const int tw = sp % a.tiles_w; sp /= a.tiles_w;
  const int th = sp % a.tiles_h; sp /= a.tiles_h;
  g.n = sp;
  PMU_DCHECK(g.n < a.in.N && g.cob_blk < a.nco, PMU_DBG_GRID);
  g.h0 = th * OH; g.w0 = tw * OW;
  g.j0 = g.cob_blk * CO;
  g.tg = wave & 3;   // tiles 16*tg .. 16*tg+15 (tile rows 2tg, 2tg+1)
  g.hh = wave >> 2;  // output channels j0 + 16*hh .. +15
  g.kk = lane >> 4;
  const int lt = 16 * g.tg + (lane & 15);
  g.pbase = (2 * (lt >> 3)) * ROWP + (2 * (lt & 7)) * LS + 2 * g.kk;
  g.ubase = (g.hh * 16 + (lane & 15)) * 4;
  return g;
}

__device__ __forceinline__ void wino_items(const WinoGeo& g, int (&ih)[NI], int (&iw)[NI], int (&dst)[NI]) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int it = threadIdx.x + NT * i;
    const int hp = it >> 2;
    const int hr = hp / HW, hc = hp - hr * HW;
    ih[i] = (it < HH * HW * 4) ? g.h0 - 1 + hr : PMU_NO_ITEM;
    iw[i] = g.w0 - 1 + hc;
    dst[i] = hr * ROWP + hc * LS + 4 * (it & 3);
  }
}

// epilogue: lane holds M[comp][tile 16*tg + 4*(lane>>4) + r][output channel j0 + 16*hh + (lane&15)]
// this lane's output-channel bias (forward); loaded before a pass's MFMAs by the multi-pass kernel
template <bool DGRAD>
__device__ __forceinline__ float wino_bias(const WinoArgs& a, const WinoGeo& g) {
  const int j = g.j0 + 16 * g.hh + (threadIdx.x & 15);
  return (!DGRAD && j < a.NOUT && a.bias) ? a.bias[j] : 0.f;
}

template <bool DGRAD>
__device__ __forceinline__ void wino_epilogue(const WinoArgs& a, const WinoGeo& g, f32x4 (&acc)[16], float* smem,
                                              float b) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const DevFrame& F = a.in;
  const int j = g.j0 + 16 * g.hh + (lane & 15);
  const bool jok = j < a.NOUT;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int t = 16 * g.tg + 4 * (lane >> 4) + r;
    const int oh = g.h0 + 2 * (t >> 3), ow = g.w0 + 2 * (t & 7);
    float m[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) m[c] = acc[c][r];
    // Y = A^T M A, A^T = [1 1 1 0; 0 1 -1 -1]
    float sr[2][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sr[0][k] = m[k] + m[4 + k] + m[8 + k];
      sr[1][k] = m[4 + k] - m[8 + k] - m[12 + k];
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const float y0 = sr[p][0] + sr[p][1] + sr[p][2] + b;
      const float y1 = sr[p][1] - sr[p][2] - sr[p][3] + b;
      const int hh = oh + p;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int ww = ow + q;
        const float y = q ? y1 : y0;
        if (!jok || hh >= F.H || ww >= F.W) continue;
        const long long pix = ((long long)g.n * F.H + hh) * F.W + ww;
        PMU_DCHECK(pix < (long long)F.N * F.H * F.W && j < a.NOUT, PMU_DBG_OUTPUT);
        if (!DGRAD) {
          a.out0[pix * a.NOUT + j] = y;
          s1 += y;
          s2 = fmaf(y, y, s2);
        } else if (j < a.split) {
          a.out0[pix * a.split + j] = y;
        } else {
          a.out1[pix * (a.NOUT - a.split) + (j - a.split)] = y;
        }
      }
    }
  }
  if (!DGRAD && a.part) {
    float* red = smem;  // [8 waves][16][2]; the last chunk's barrier freed the stage
    s1 += __shfl_xor(s1, 16, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (lane < 16) {
      red[(wave * 16 + lane) * 2 + 0] = s1;
      red[(wave * 16 + lane) * 2 + 1] = s2;
    }
    __syncthreads();
    if (tid < CO) {  // channel tid: half tid >> 4, summed over the 4 tile groups (waves 4*half + tg)
      const int jj = g.j0 + tid, hf = tid >> 4, l = tid & 15;
      if (jj < a.NOUT) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int tg = 0; tg < 4; ++tg) {
          t1 += red[((4 * hf + tg) * 16 + l) * 2 + 0];
          t2 += red[((4 * hf + tg) * 16 + l) * 2 + 1];
        }
        PMU_DCHECK(g.spatial < (long long)F.N * a.tiles_h * a.tiles_w, PMU_DBG_WORKSPACE);
        a.part[((long long)g.spatial * 2 + 0) * a.NOUT + jj] = t1;
        a.part[((long long)g.spatial * 2 + 1) * a.NOUT + jj] = t2;
      }
    }
  }
}

// synchronous staging (any frame): stage, barrier, MFMAs, barrier
template <bool DGRAD>
__global__ __launch_bounds__(NT, 1) void conv3x3_wino_kernel(WinoArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[A_FLOATS + U_FLOATS];
  float* As = smem;
  float* Us = smem + A_FLOATS;
  const int tid = threadIdx.x;
  const WinoGeo g = wino_geo(a);
  const DevFrame& F = a.in;
  const int nchunks = (a.KC + BK - 1) / BK;
  int ih[NI], iw[NI], dst[NI];
  wino_items(g, ih, iw, dst);
  f32x4 acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float4* wsrc = reinterpret_cast<const float4*>(a.wp + (long long)g.cob_blk * nchunks * U_FLOATS);
  for (int ch = 0; ch < nchunks; ++ch) {
    const int k0 = ch * BK;
#pragma unroll 1
    for (int i = 0; i < NI; ++i)  // generic staging: this kernel takes the frames the pipelined one does not
      if (ih[i] != PMU_NO_ITEM) *reinterpret_cast<float4*>(As + dst[i]) = frame_value4(F, g.n, ih[i], iw[i], k0 + 4 * (tid & 3));
    {
      const float4* s = wsrc + (long long)ch * (U_FLOATS / 4);
#pragma unroll
      for (int r = 0; r < U_FLOATS / 4 / NT; ++r) reinterpret_cast<float4*>(Us)[tid + NT * r] = s[tid + NT * r];
    }
    __syncthreads();
    if (a.tee && g.cob_blk == 0) wino_tee(a, As, k0, g.n, g.h0, g.w0, tid);
    wino_chunk(As, Us, g.pbase, g.ubase, g.kk, acc);
    __syncthreads();
  }
  wino_epilogue<DGRAD>(a, g, acc, smem, wino_bias<DGRAD>(a, g));
}

// Software-pipelined variant (the default for fast-path frames): the next chunk's operand items and
// U tile are loaded into registers before this chunk's MFMAs and written to the other LDS stage after
// them — one barrier per chunk; 1 block (8 waves, 2 per SIMD) per CU, 118 KB LDS.
constexpr int STAGE = A_FLOATS + U_FLOATS;
static_assert(U_FLOATS / 4 / NT == 4, "4 U float4 (LDS-DMA) per thread per chunk");

// EXP (timing experiments, PMU_WINO_EXP): 1 = no restaging (every chunk reuses the first), 2 = that
// and no barrier, 3 = no input transform, 6 = no U restaging, 7 = no operand restaging (results wrong
// for 1-3, 6, 7); 4 / 5 = commit in step 1 / 3 instead of 2 (correct).
template <bool DGRAD, int POOL, int EXP = 0>
__global__ __launch_bounds__(NT, 1) void conv3x3_wino_pipe_kernel(WinoArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x;
  const WinoGeo g = wino_geo(a);
  const DevFrame& F = a.in;
  const int nchunks = (a.KC + BK - 1) / BK;
  const int cq4 = 4 * (tid & 3);
  int ih[NI], iw[NI], dst[NI];
  wino_items(g, ih, iw, dst);
  f32x4 acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};

  PmuPref<POOL, DGRAD, NI> pf;
  // U is a plain copy: global_load_lds (LDS-DMA, no registers) straight into the stage, in the
  // global layout (wave-instruction = 1 KB contiguous)
  const float* wsrc = a.wp + (long long)g.cob_blk * nchunks * U_FLOATS + 4 * tid;
  const int wave_off = (tid >> 6) * 256;  // floats: this wave's 1 KB within each 8 KB row of 512 float4
#define PMU_WPREFETCH(CH, BUF)                                                                              \
  {                                                                                                        \
    const int k0_ = (CH) * BK;                                                                             \
    const bool second_ = F.nsrc > 1 && k0_ >= F.C0;                                                        \
    if (EXP != 7)                                                                                          \
      pmu_prefetch<POOL, DGRAD, NI>(pmu_pick_src(F, second_), k0_ - (second_ ? F.C0 : 0) + cq4, g.n, ih, iw, pf); \
    const float* s_ = wsrc + (long long)(CH) * U_FLOATS;                                                   \
    float* d_ = (BUF) + A_FLOATS + wave_off;                                                               \
    if (EXP != 6) {                                                                                        \
      PMU_GLDS(s_, d_) PMU_GLDS(s_ + 4 * NT, d_ + 4 * NT) PMU_GLDS(s_ + 8 * NT, d_ + 8 * NT)               \
      PMU_GLDS(s_ + 12 * NT, d_ + 12 * NT)                                                                 \
    }                                                                                                      \
  }
#define PMU_GLDS(S, D)                                                                                      \
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(S),                     \
                                   (__attribute__((address_space(3))) void*)(D), 16, 0, 0);
#define PMU_WCOMMIT(BUF) if (EXP != 7) pmu_commit<POOL, DGRAD, NI>(pf, ih, dst, (BUF));
  PMU_WPREFETCH(0, smem)
  PMU_WCOMMIT(smem)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int ch = 0; ch < nchunks; ++ch) {
    float* cur = smem + (ch & 1) * STAGE;
    if (EXP == 1 || EXP == 2) cur = smem;
    if (ch + 1 < nchunks && EXP != 1 && EXP != 2) PMU_WPREFETCH(ch + 1, smem + ((ch + 1) & 1) * STAGE)
    if (a.tee && g.cob_blk == 0) wino_tee(a, cur, ch * BK, g.n, g.h0, g.w0, tid);
    {
      // wino_chunk with the next chunk's LDS stores issued inside step CS: they drain under this
      // chunk's MFMAs instead of in a store phase all waves of the block would enter together
      // (BN-backward and max-pool operands hold more prefetch registers: they commit after the steps)
      constexpr int CS = EXP == 4 ? 1 : EXP == 5 ? 3 : (DGRAD || POOL != PMU_POOL_NONE) ? 4 : 2;
      const bool commit = ch + 1 < nchunks && EXP != 1 && EXP != 2;
      const unsigned pa = lds_addr(cur + g.pbase);
      const unsigned ua = lds_addr(cur + A_FLOATS + g.ubase) + (unsigned)(2 * g.kk * 4 * CO * 4 * 4);
      float2 dp[2][16];
      float4 u[2][4];
      wino_load_patch(pa, dp[0]);
      wino_load_u(ua, u[0]);
#pragma unroll
      for (int ks = 0; ks < BK / 4; ++ks) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (ks + 1 < BK / 4) {
          const int n1 = ks + 1;
          if ((n1 & 1) == 0) wino_load_patch(pa + 32 * (n1 >> 1), dp[(n1 >> 1) & 1]);
          wino_load_u(ua + (unsigned)((8 * (n1 >> 1) + (n1 & 1)) * 4 * CO * 4 * 4), u[n1 & 1]);
        }
        if (ks == CS && commit) PMU_WCOMMIT(smem + ((ch + 1) & 1) * STAGE)
        __builtin_amdgcn_sched_barrier(0);
        wino_mfmas<EXP == 3>(dp[(ks >> 1) & 1], ks & 1, u[ks & 1], acc);
        __builtin_amdgcn_sched_barrier(0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (CS == 4 && commit) PMU_WCOMMIT(smem + ((ch + 1) & 1) * STAGE)
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA of the next U has landed
    if (EXP != 2) __syncthreads();
  }
#undef PMU_WPREFETCH
#undef PMU_WCOMMIT
#undef PMU_GLDS
  wino_epilogue<DGRAD>(a, g, acc, smem, wino_bias<DGRAD>(a, g));
}

#ifdef PMU_EXPERIMENTS
// (the 512-thread raw kernels: superseded by the 1024-thread conv3x3_wino2h.hip kernels on every shape
// they take; experiments build only, PMU_WINO2H=0 A/B)
// ---------------------------------------------------------------------------------------------
// RAW-operand variant: the operand was materialised once (BN+ReLU / pool /
// F.pad+cat applied, or the BN backward of dz) — the tensor the weight gradient reads anyway — so
// the staging is a copy done by LDS-DMA (global_load_lds, no registers, no VALU), and each lane reads
// its 4x4 patch once per chunk as 16 ds_read_b128 (4 channels: channel 4*kk + ks feeds step ks).
// Halo rows are RROWP = 384 floats (2*RROWP = 0 mod 64), pixels 20 floats: with the tile/lane map
// the b128 patch reads are conflict-free.  Units of the image outside the input are zeroed once
// (their DMA lanes are masked), pad units are never written.
// ---------------------------------------------------------------------------------------------
constexpr int RROWP = 384;
constexpr int R_A_FLOATS = HH * RROWP;
constexpr int R_STAGE = R_A_FLOATS + U_FLOATS;
constexpr int R_UNITS = R_A_FLOATS / 4;           // 16-B units of the operand image (data + pads)
constexpr int R_NGL = (R_UNITS + NT - 1) / NT;    // operand DMA instructions per thread per chunk
static_assert(R_NGL == 4, "operand image of 4 DMA rounds");

// MULTI: the workgroup walks a.cpb output-channel blocks in passes (the K-short 64-channel layers
// lose most to the per-workgroup prologue).  The forward's bias is loaded before each pass's MFMAs:
// loaded in the epilogue, the compiler waited vmcnt(0) on the next pass's in-flight DMAs at the
// next register reuse, and the forward measured 14% slower as a multi-pass kernel.
template <bool DGRAD, bool MULTI>
__global__ __launch_bounds__(NT, 1) void conv3x3_wino_raw_kernel(WinoArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * R_STAGE + 8 * 16 * 2];
  float* red = smem + 2 * R_STAGE;  // the epilogue's BN partials (kept apart: a DMA may be in flight)
  const int tid = threadIdx.x, lane = tid & 63;
  const WinoGeo g = wino_geo(a);
  const DevFrame& F = a.in;
  const float* x = F.s0.x;
  const int KC = a.KC;
  const int nchunks = KC / BK;

  // this thread's operand units: global BYTE offset (chunk 0; < 2^32, host-checked) and whether
  // the unit is inside the input.  The DMA addresses are a uniform base (SGPRs) plus these 32-bit
  // offsets, so the loop issues them in global_load_lds's saddr form and writes no address VGPRs.
  unsigned goff[R_NGL];
  unsigned gin = 0u;
#pragma unroll
  for (int r = 0; r < R_NGL; ++r) {
    const int u = r * NT + tid;
    const int hr = u / (RROWP / 4), wu = u - hr * (RROWP / 4);
    const int hc = wu / 5, q = wu - hc * 5;
    const bool data = u < R_UNITS && q < 4 && hc < HW;
    const int h = g.h0 - 1 + hr, w = g.w0 - 1 + hc;
    const bool in = data && h >= 0 && w >= 0 && h < F.H && w < F.W;
    goff[r] = in ? (unsigned)(((((long long)g.n * F.H + h) * F.W + w) * KC + 4 * q) * 4) : 0u;
    PMU_DCHECK(!in || (((long long)g.n * F.H + h) * F.W + w) < (long long)F.N * F.H * F.W, PMU_DBG_OPERAND);
    gin |= in ? (1u << r) : 0u;
    if (data && !in) {  // zero padding, in both stages, once
      *reinterpret_cast<float4*>(smem + 4 * u) = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(smem + R_STAGE + 4 * u) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // passes over this block's output-channel blocks: the flat chunk sequence (pass, chunk) is one
  // pipeline, so the next pass's first operand image and U tile arrive under this pass's last MFMAs
  const int npass = !MULTI ? 1 : a.cpb < a.nco - g.cob_blk ? a.cpb : a.nco - g.cob_blk;
  const int total = npass * nchunks;
  const float* wsrc = a.wp + (long long)g.cob_blk * nchunks * U_FLOATS;  // uniform
  const unsigned uoff = 16u * tid;
  const int wave_off = (tid >> 6) * 256;
#define PMU_GLDS(S, D)                                                                                      \
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(S),                     \
                                   (__attribute__((address_space(3))) void*)(D), 16, 0, 0);
#define PMU_RFETCH(GI, BUF)                                                                                 \
  {                                                                                                        \
    const int p_ = (GI) / nchunks;                                                                         \
    const int k0_ = ((GI) - p_ * nchunks) * BK;                                                            \
    PMU_DCHECK(k0_ + BK <= KC, PMU_DBG_OPERAND);                                                           \
    float* b_ = (BUF);                                                                                     \
    const char* xb_ = reinterpret_cast<const char*>(x + k0_);                                              \
    for (int r = 0; r < R_NGL; ++r)                                                                        \
      if ((gin >> r) & 1u) PMU_GLDS(xb_ + goff[r], b_ + 4 * (r * NT) + wave_off)                           \
    /* pass p_ = co-block cob_blk + p_ */                                                                  \
    const char* s_ = reinterpret_cast<const char*>(wsrc + (long long)(GI) * U_FLOATS) + uoff;              \
    float* d_ = b_ + R_A_FLOATS + wave_off;                                                                \
    PMU_GLDS(s_, d_) PMU_GLDS(s_ + 16 * NT, d_ + 4 * NT) PMU_GLDS(s_ + 32 * NT, d_ + 8 * NT)               \
    PMU_GLDS(s_ + 48 * NT, d_ + 12 * NT)                                                                   \
  }
  f32x4 acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int lt = 16 * g.tg + (lane & 15);
  const int pbase = (2 * (lt >> 3)) * RROWP + (2 * (lt & 7)) * LS + 4 * g.kk;
  if (a.prio && (tid >> 6) >= 4) __builtin_amdgcn_s_setprio(1);  // the younger half wins VALU arbitration
  PMU_RFETCH(0, smem)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int p = 0; p < npass; ++p) {
  // the pass's bias, loaded before its MFMAs (a load issued in the epilogue made the compiler
  // wait vmcnt(0) — on the next pass's in-flight DMAs — at the next register reuse)
  WinoGeo gp = g;
  gp.cob_blk = g.cob_blk + p;
  gp.j0 = gp.cob_blk * CO;
  const float bias_p = wino_bias<DGRAD>(a, gp);
  for (int ch = 0; ch < nchunks; ++ch) {
    const int gi = p * nchunks + ch;
    float* cur = smem + (gi & 1) * R_STAGE;
    if (gi + 1 < total) PMU_RFETCH(gi + 1, smem + ((gi + 1) & 1) * R_STAGE)
    const unsigned pa = lds_addr(cur + pbase);
    // U of step ks for this lane: channel 4*kk + ks
    const unsigned ua = lds_addr(cur + R_A_FLOATS + g.ubase) + (unsigned)(4 * g.kk * 4 * CO * 4 * 4);
    float4 pt[16];
#define PMU_P(I, J) pt[4 * I + J] = lds_b128<((I) * RROWP + (J) * LS) * 4>(pa);
    PMU_P(0, 0) PMU_P(0, 1) PMU_P(0, 2) PMU_P(0, 3) PMU_P(1, 0) PMU_P(1, 1) PMU_P(1, 2) PMU_P(1, 3)
    PMU_P(2, 0) PMU_P(2, 1) PMU_P(2, 2) PMU_P(2, 3) PMU_P(3, 0) PMU_P(3, 1) PMU_P(3, 2) PMU_P(3, 3)
#undef PMU_P
    float4 u[2][4];
    wino_load_u(ua, u[0]);
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (ks + 1 < BK / 4) wino_load_u(ua + (unsigned)((ks + 1) * 4 * CO * 4 * 4), u[(ks + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      float dd[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 t = pt[4 * i + j];
          dd[i][j] = ks == 0 ? t.x : ks == 1 ? t.y : ks == 2 ? t.z : t.w;
        }
      float v[16];
      input_transform(dd, v);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const float4 uu = u[ks & 1][gq];
        acc[4 * gq + 0] = mfma16(v[4 * gq + 0], uu.x, acc[4 * gq + 0]);
        acc[4 * gq + 1] = mfma16(v[4 * gq + 1], uu.y, acc[4 * gq + 1]);
        acc[4 * gq + 2] = mfma16(v[4 * gq + 2], uu.z, acc[4 * gq + 2]);
        acc[4 * gq + 3] = mfma16(v[4 * gq + 3], uu.w, acc[4 * gq + 3]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next chunk's DMA has landed
    __syncthreads();
  }
    // end of a pass: this co-block's output
    wino_epilogue<DGRAD>(a, gp, acc, red, bias_p);
    if (MULTI) {
#pragma unroll
      for (int c = 0; c < 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
#undef PMU_RFETCH
#undef PMU_GLDS
}

int launch_wino_raw(const float* x, int KC, int N, int H, int W, const float* wp, const float* bias, int NOUT,
                    float* out0, float* out1, int split, float* part, bool dgrad, void* stream) {
  PMU_REQUIRE(x && wp && out0 && KC > 0 && KC % BK == 0 && NOUT > 0 && N > 0 && H > 0 && W > 0);
  const long long img_bytes = (long long)H * W * (KC > NOUT ? KC : NOUT) * 4;
  if ((long long)N * img_bytes >= (1LL << 32)) {  // 32-bit DMA byte offsets: split over images
    const long long tiles = (long long)pmu_cdiv(W, OW) * pmu_cdiv(H, OH);
    return pmu_image_chunks(N, img_bytes, [&](int n0, int nn) {
      const long long px = (long long)n0 * H * W;
      return launch_wino_raw(x + px * KC, KC, nn, H, W, wp, bias, NOUT, out0 + px * split,
                  out1 ? out1 + px * (NOUT - split) : nullptr, split,
                  part ? part + (long long)n0 * tiles * 2 * NOUT : nullptr, dgrad, stream);
    });
  }
  WinoArgs a;
  memset(&a, 0, sizeof(a));
  a.in.s0.x = x; a.in.s0.C = KC; a.in.s0.H = H; a.in.s0.W = W;
  a.in.nsrc = 1; a.in.N = N; a.in.H = H; a.in.W = W; a.in.C0 = KC; a.in.C = KC; a.in.vec = 1;
  a.wp = wp; a.bias = bias; a.out0 = out0; a.out1 = out1; a.part = part; a.tee = nullptr;
  a.NOUT = NOUT; a.KC = KC; a.split = split;
  a.tiles_w = pmu_cdiv(W, OW);
  a.tiles_h = pmu_cdiv(H, OH);
  a.nco = pmu_cdiv(NOUT, CO);
  static const int prio = [] {  // PMU_WINO_PRIO=0|1 (A/B of static wave priority)
    const char* e = pmu_variant_env("PMU_WINO_PRIO");
    return e ? atoi(e) : 0;
  }();
  a.prio = prio;
  // co-block passes per workgroup: fewer, longer workgroups (the prologue of all but the first pass
  // hides under MFMAs) while keeping >= 8 workgroups per CU; PMU_WINO_CPB forces a value (A/B)
  static const int cpb_env = [] {
    const char* e = getenv("PMU_WINO_CPB");
    return e ? atoi(e) : 0;
  }();
  const long long spatial = (long long)a.tiles_w * a.tiles_h * N;
  static const bool fwd_multi = [] {  // PMU_WINO_FWD_MULTI=0: one pass per forward workgroup (A/B)
    const char* e = pmu_variant_env("PMU_WINO_FWD_MULTI");
    return !(e && atoi(e) == 0);
  }();
  int cpb = 1;
  if (!dgrad && !fwd_multi) {
    // one pass (see MULTI)
  } else if (cpb_env > 0) {
    cpb = cpb_env < a.nco ? cpb_env : a.nco;
  } else {
    static const long long min_wg = [] {  // PMU_WINO_MINWG: fewest workgroups the passes may leave
      const char* e = getenv("PMU_WINO_MINWG");
      return e ? atoll(e) : 1024LL;
    }();
    while (cpb * 2 <= a.nco && spatial * pmu_cdiv(a.nco, cpb * 2) >= min_wg) cpb *= 2;
  }
  a.cpb = cpb;
  const long long blocks = (long long)pmu_cdiv(a.nco, cpb) * spatial;
  PMU_REQUIRE(blocks < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  if (dgrad) hipLaunchKernelGGL((conv3x3_wino_raw_kernel<true, true>), dim3((unsigned)blocks), dim3(NT), 0, st, a);
  else if (fwd_multi) hipLaunchKernelGGL((conv3x3_wino_raw_kernel<false, true>), dim3((unsigned)blocks), dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((conv3x3_wino_raw_kernel<false, false>), dim3((unsigned)blocks), dim3(NT), 0, st, a);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
#endif  // PMU_EXPERIMENTS

// a source the pipelined staging takes: float4 channels, chunks never straddle sources
static bool wino_pipe_src_ok(const pmu_src& s) {
  if (s.C % BK != 0) return false;
  if (s.pool == PMU_POOL_NONE) return true;
  return (s.pool == PMU_POOL_MAX2 || s.pool == PMU_POOL_AVG2CEIL) && s.mode == PMU_SRC_BNRELU;
}

#ifdef PMU_EXPERIMENTS
// timing experiments (EXP 1-3, 6, 7 compute wrong results): only in `make EXPERIMENTS=1` builds
static int wino_exp() {
  static const int v = [] {
    const char* e = pmu_variant_env("PMU_WINO_EXP");
    return e ? atoi(e) : 0;
  }();
  return v;
}
#endif

static bool wino_sync_forced() {
  static const bool v = [] {
    const char* e = pmu_variant_env("PMU_WINO_IMPL");
    return e && strcmp(e, "sync") == 0;
  }();
  return v;
}

int launch_wino(const pmu_frame* in, const float* wp, const float* bias, int NOUT, int KC, float* out0, float* out1,
                int split, float* part, float* tee, bool dgrad, void* stream) {
  WinoArgs a;
  a.prio = 0;
  a.cpb = 1;
  a.in = make_dev_frame(in);
  a.wp = wp; a.bias = bias; a.out0 = out0; a.out1 = out1; a.part = part; a.tee = tee;
  a.NOUT = NOUT; a.KC = KC; a.split = split;
  a.tiles_w = pmu_cdiv(in->W, OW);
  a.tiles_h = pmu_cdiv(in->H, OH);
  a.nco = pmu_cdiv(NOUT, CO);
  const long long blocks = (long long)a.nco * a.tiles_w * a.tiles_h * in->N;
  PMU_REQUIRE(blocks < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)blocks);
  if (!wino_sync_forced()) {
    const pmu_src& s0 = in->src[0];
    const bool two = in->nsrc > 1;
    const bool ok = wino_pipe_src_ok(s0) && (!two || wino_pipe_src_ok(in->src[1]));
    const int pool = s0.pool;
    const bool same_pool = !two || in->src[1].pool == pool;
    const bool modes_ok = dgrad ? (!two && s0.mode == PMU_SRC_BNBWD)
                                : (s0.mode != PMU_SRC_BNBWD && (!two || in->src[1].mode != PMU_SRC_BNBWD));
    if (ok && same_pool && modes_ok) {
      if (dgrad && pool == PMU_POOL_NONE)
        hipLaunchKernelGGL((conv3x3_wino_pipe_kernel<true, PMU_POOL_NONE>), grid, dim3(NT), 0, st, a);
#ifdef PMU_EXPERIMENTS
      else if (!dgrad && pool == PMU_POOL_NONE && wino_exp() == 1)
        hipLaunchKernelGGL((conv3x3_wino_pipe_kernel<false, PMU_POOL_NONE, 1>), grid, dim3(NT), 0, st, a);
      else if (!dgrad && pool == PMU_POOL_NONE && wino_exp() == 2)
        hipLaunchKernelGGL((conv3x3_wino_pipe_kernel<false, PMU_POOL_NONE, 2>), grid, dim3(NT), 0, st, a);
      else if (!dgrad && pool == PMU_POOL_NONE && wino_exp() == 3)
        hipLaunchKernelGGL((conv3x3_wino_pipe_kernel<false, PMU_POOL_NONE, 3>), grid, dim3(NT), 0, st, a);
      else if (!dgrad && pool == PMU_POOL_NONE && wino_exp() == 4)
        hipLaunchKernelGGL((conv3x3_wino_pipe_kernel<false, PMU_POOL_NONE, 4>), grid, dim3(NT), 0, st, a);
      else if (!dgrad && pool == PMU_POOL_NONE && wino_exp() == 5)
        hipLaunchKernelGGL((conv3x3_wino_pipe_kernel<false, PMU_POOL_NONE, 5>), grid, dim3(NT), 0, st, a);
      else if (!dgrad && pool == PMU_POOL_NONE && wino_exp() == 6)
        hipLaunchKernelGGL((conv3x3_wino_pipe_kernel<false, PMU_POOL_NONE, 6>), grid, dim3(NT), 0, st, a);
      else if (!dgrad && pool == PMU_POOL_NONE && wino_exp() == 7)
        hipLaunchKernelGGL((conv3x3_wino_pipe_kernel<false, PMU_POOL_NONE, 7>), grid, dim3(NT), 0, st, a);
#endif
      else if (!dgrad && pool == PMU_POOL_NONE)
        hipLaunchKernelGGL((conv3x3_wino_pipe_kernel<false, PMU_POOL_NONE>), grid, dim3(NT), 0, st, a);
      else if (!dgrad && pool == PMU_POOL_MAX2)
        hipLaunchKernelGGL((conv3x3_wino_pipe_kernel<false, PMU_POOL_MAX2>), grid, dim3(NT), 0, st, a);
      else if (!dgrad && pool == PMU_POOL_AVG2CEIL)
        hipLaunchKernelGGL((conv3x3_wino_pipe_kernel<false, PMU_POOL_AVG2CEIL>), grid, dim3(NT), 0, st, a);
      else
        goto sync;
      PMU_CHECK_LAUNCH();
      return PMU_OK;
    }
  }
sync:
  if (dgrad) hipLaunchKernelGGL((conv3x3_wino_kernel<true>), dim3((unsigned)blocks), dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((conv3x3_wino_kernel<false>), dim3((unsigned)blocks), dim3(NT), 0, st, a);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

}  // namespace

extern "C" int pmu_conv3x3_tiles_wino(int N, int H, int W) { return N * pmu_cdiv(H, OH) * pmu_cdiv(W, OW); }

extern "C" size_t pmu_conv3x3_packed_size_wino(int Cout, int Cin, int dgrad) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  return (size_t)pmu_cdiv(NOUT, CO) * pmu_cdiv(KC, BK) * U_FLOATS * sizeof(float);
}

extern "C" int pmu_conv3x3_pack_wino(const float* w, int Cout, int Cin, int dgrad, float* wp, void* stream) {
  PMU_REQUIRE(w && wp && Cout > 0 && Cin > 0);
  const long long total = (long long)pmu_conv3x3_packed_size_wino(Cout, Cin, dgrad) / sizeof(float) / 16;
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  hipLaunchKernelGGL(pack_wino_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, dgrad, wp);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_conv3x3_fwd_wino(const pmu_frame* in, const float* wp, const float* bias, int Cout, float* z,
                                    float* part, float* tee, void* stream) {
  PMU_REQUIRE(valid_frame(in) && wp && z && Cout > 0);
  const int Cin = in->src[0].C + (in->nsrc > 1 ? in->src[1].C : 0);
  PMU_REQUIRE(!tee || Cin % 4 == 0);
  return launch_wino(in, wp, bias, Cout, Cin, z, nullptr, Cout, part, tee, false, stream);
}

extern "C" int pmu_conv3x3_dgrad_wino(const pmu_frame* dz, const float* wp, int Cin, int Csplit, float* dx0, float* dx1,
                                      float* tee, void* stream) {
  PMU_REQUIRE(valid_frame(dz) && dz->nsrc == 1 && wp && dx0 && Cin > 0);
  PMU_REQUIRE(Csplit > 0 && Csplit <= Cin && (Csplit == Cin || dx1));
  const int Cout = dz->src[0].C;
  PMU_REQUIRE(!tee || Cout % 4 == 0);
  return launch_wino(dz, wp, nullptr, Cin, Cout, dx0, dx1, Csplit, nullptr, tee, true, stream);
}

#ifdef PMU_EXPERIMENTS
extern "C" int pmu_conv3x3_fwd_wino_raw(const float* xt, int Cin, int N, int H, int W, const float* wp,
                                        const float* bias, int Cout, float* z, float* part, void* stream) {
  return launch_wino_raw(xt, Cin, N, H, W, wp, bias, Cout, z, nullptr, Cout, part, false, stream);
}

extern "C" int pmu_conv3x3_dgrad_wino_raw(const float* dzt, int Cout, int N, int H, int W, const float* wp, int Cin,
                                          int Csplit, float* dx0, float* dx1, void* stream) {
  PMU_REQUIRE(Csplit > 0 && Csplit <= Cin && (Csplit == Cin || dx1));
  return launch_wino_raw(dzt, Cout, N, H, W, wp, nullptr, Cin, dx0, dx1, Csplit, nullptr, true, stream);
}
#endif  // PMU_EXPERIMENTS

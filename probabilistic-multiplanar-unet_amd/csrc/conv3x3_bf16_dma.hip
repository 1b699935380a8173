// 3x3 / pad 1 convolution of a materialised bf16 NHWC operand on bf16 MFMA, both operands staged by
// LDS-DMA: config c5's forward and input gradient (nn.Conv2d at PMU/model/unet/unet_parts.py:15,18
// under torch.autocast(bfloat16)), for maps at least 32 pixels wide.
//
// GEMM view per workgroup: BM output pixels (a TH x 32 tile of one image) x BN output channels, K =
// 9 taps x channels in chunks of 16 (one v_mfma_f32_32x32x16_bf16 k-step per tap).  Per chunk the
// (TH+2) x 34 halo image (16 channels) and the chunk's 9 x BN x 16 packed weights arrive by
// global_load_lds (16 B per lane) in one of two LDS stages while the other stage feeds the MFMAs: no
// staging registers, no ds_write, no transform.  The halo image serves all 9 taps from LDS.
//
// A wave owns 128 pixels (4 tile rows = 4 32-row fragments) x 64 channels (2 32-column fragments): 8
// accumulators of 16, 6 ds_read_b128 per 8 MFMAs, ~236 VGPRs (two waves per SIMD).  Two workgroup
// shapes (dma_shape): 512 pixels x 128 channels in 8 waves (one workgroup per CU), and 512 pixels x
// 64 channels in 4 waves (two per CU) for <= 64 output channels or reductions of <= 128 channels.
//
// LDS-DMA writes each wave-instruction's 64 x 16 B contiguously, so the conflict-free layout is a
// permutation of 16-B units, not a padded row: unit (pixel p, channel half q) sits at 2p + (q XOR
// bit 3 of p).  A 32-lane fragment read (32 consecutive pixels, one half) then hits 16 distinct
// 4-bank groups in each ds_read_b128 lane group, for any starting pixel (every tap).  The weights are
// packed in the same order (channel co in place of the pixel), so their DMA is a straight copy.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "pmu_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BK = 16;              // channels per chunk
constexpr int TW = 32, HW2 = 34;    // tile width (one 32-pixel fragment per tile row), halo width

// NWV waves per workgroup (8: one workgroup per CU; 4: two per CU, one's prologue / epilogue under
// the other's MFMAs), WN of them across the BN = 64 WN output channels
template <int WN, int NWV>
struct DG {
  static constexpr int NT = 64 * NWV;
  static constexpr int BN = 64 * WN;
  static constexpr int WM = NWV / WN;
  static constexpr int TH = 4 * WM;
  static constexpr int HP = (TH + 2) * HW2;
  static constexpr int A_UNITS = 2 * HP;
  static constexpr int B_UNITS = 18 * BN;       // 9 taps x BN channels x 2 halves
  static constexpr int NGA = (A_UNITS + NT - 1) / NT;
  static constexpr int NGB = (B_UNITS + NT - 1) / NT;
  static constexpr int A_BYTES = 16 * A_UNITS;
  static constexpr int STAGE = A_BYTES + 16 * B_UNITS;
  static_assert(2 * STAGE <= 160 * 1024, "LDS");
  static_assert(NGA <= 8, "gin / gzero masks");
};

struct DmaArgs {
  const unsigned short* x;   // operand [N][H][W][Cp] bf16
  const unsigned short* wp;  // packed [co block][chunk][tap][unit][8] bf16
  const float* bias;
  float* out0;
  float* out1;
  unsigned short* out1b;  // input gradient, nullable: a bf16 (RNE) copy of out1 (the convT's bf16 operand)
  float* part;
  int N, H, W, Cp, NOUT, split, tiles_w, tiles_h, nch, ncb;
  // input gradient only: the producer layer's BatchNorm+ReLU backward partial sums (see
  // pmu_conv3x3_dgrad_wino4_bnr); null: none
  const float* bz;
  const float* bcoef;
  const float* bmean;
  const float* binv;
  // bf16 z (torch.autocast's conv output dtype), centred: forward — z stored as bf16(z - zoff[c]) (RNE;
  // zoff = the BN's running mean, so the stored value keeps bf16's relative precision against the
  // channel's spread, not its mean) and the BN partial sums taken over the stored values + zoff;
  // input gradient — bz holds such values (its consumer passes the correspondingly shifted coef/mean)
  int zbf;
  const float* zoff;
};

__device__ __forceinline__ int swz(int p, int q) { return 2 * p + (q ^ ((p >> 3) & 1)); }

// Output stores that do not stay in the XCD's L2 (relaxed agent-scope atomic stores: `sc1`, written
// through and dropped): z / dx are next read by another kernel, long after they would have left L2,
// and kept lines evict the operand halo that the next chunks of the resident tiles re-read.
__device__ __forceinline__ void st_drop(float* p, float2 v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_drop(unsigned short* p, unsigned v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned short bf16_bits(float v) { return __builtin_bit_cast(unsigned short, (__bf16)v); }

// wp[jb][ch][tap][u][e]: unit u = swz(co, q) holds B[tap][k = 16 ch + 8 q + e][j = BN jb + co], zero
// padded, bf16 RNE.  Forward: B[tap][ci][co] = w[co][ci][tap]; dgrad: B[tap][co][ci] = w[co][ci][8 - tap].
__device__ __forceinline__ void pack_dma_body(const float* __restrict__ w, int Cout, int Cin, int dgrad, int BN,
                                              unsigned short* __restrict__ wp, int bid, int nblk) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  const int nch = (KC + BK - 1) / BK, njb = (NOUT + BN - 1) / BN;
  const long long total = (long long)njb * nch * 9 * 2 * BN * 8;
  for (long long e = (long long)bid * blockDim.x + threadIdx.x; e < total; e += (long long)nblk * blockDim.x) {
    const int el = (int)(e & 7);
    long long r = e >> 3;
    const int u = (int)(r % (2 * BN)); r /= 2 * BN;
    const int tap = (int)(r % 9); r /= 9;
    const int ch = (int)(r % nch);
    const int jb = (int)(r / nch);
    const int co = u >> 1, q = (u & 1) ^ ((co >> 3) & 1);
    const int j = jb * BN + co, k = ch * BK + 8 * q + el;
    float v = 0.f;
    if (j < NOUT && k < KC)
      v = dgrad ? w[((long long)k * Cin + j) * 9 + (8 - tap)] : w[((long long)j * Cin + k) * 9 + tap];
    wp[e] = bf16_bits(v);
  }
}
__global__ __launch_bounds__(256) void pack_dma_kernel(const float* __restrict__ w, int Cout, int Cin, int dgrad, int BN,
                                                       unsigned short* __restrict__ wp) {
  pack_dma_body(w, Cout, Cin, dgrad, BN, wp, blockIdx.x, gridDim.x);
}
// workgroup channel width of a conv (see dma_shape): 64 for <= 64 outputs or a <= 128-channel reduction
__host__ __device__ __forceinline__ int dma_bn(int NOUT, int KC) {
  return (NOUT <= 64 || (KC + BK - 1) / BK * BK <= 128) ? 64 : 128;
}
__global__ __launch_bounds__(256) void pack_dma_multi_kernel(const pmu_pack_job* __restrict__ jobs, int njobs, int dgrad) {
  const pmu_pack_job& j = jobs[pmu_job_of(jobs, njobs, blockIdx.x)];
  const int NOUT = dgrad ? j.Cin : j.Cout, KC = dgrad ? j.Cout : j.Cin;
  pack_dma_body(j.w, j.Cout, j.Cin, dgrad, dma_bn(NOUT, KC), (unsigned short*)j.dst, blockIdx.x - j.block0, j.nblocks);
}

// ZB: z stored in bf16 (the experiments-build bf16-z mode: the forward writes it, the input gradient's
// BN-backward epilogue reads it)
// EXP (timing experiments, experiments build only, PMU_DMA_EXP; wrong results on purpose): bit 0 = no
// epilogue output stores, bit 1 = no MFMAs.  512^2 x 64 -> 64 (c5, tools/kbench.py --c5): 0.52 ms; no
// stores 0.33; no MFMAs 0.36; neither 0.17 — the z stores (1.07 GB fp32) and the MFMAs add up instead
// of overlapping.  Measured and dropped: a phase offset between the two workgroups of a CU (s_sleep
// before the first round: no change), 16-B stores through an LDS transpose (-2..5% on K <= 128
// only), and the transposed accumulator layout (MFMA operands swapped: a pixel per lane, four
// consecutive channels per register group, so every z / dx store and the BN-backward z loads are
// 16 B and bf16 dx leaves in permlane32-swapped 16-B vectors — a quarter of the store instructions;
// BN sums through LDS): kbench --c5 fwd 4.57 vs 4.42 ms, dgrad_bnr 6.44 vs 5.92 (profiles/r05/
// transposed_epilogue) — the store tail here is not issue-bound.
// CS (input gradient): per-tile column sums of dx into a.part instead of the BN-backward partials
// (pmu_conv3x3_dgrad_dma_x1b_sum; a compile-time variant: as a runtime branch beside the a.bz one it
// spilled 89 VGPRs)
// XB (input gradient, the *_dxb entries): dx rounded to bf16 (RNE) as torch.autocast's conv backward
// returns it, before anything is formed from it — dx0 stored as bf16 (out0 holds 2-byte values), dx1
// (fp32 storage, when requested) holding the rounded values, the bf16 copy, column sums and the
// producer's BN-backward partials all taken from the rounded values.  Halves the bytes of the
// activation-gradient stream its consumers (the BN-backward dz stream, the max-pool backward, the
// first layer's weight gradient) read.
// PERS (persistent): one resident workgroup per slot walks a run of tiles of one channel block (its
// XCD's share of the tiles, interleaved with the other slots of that XCD): the next tile's chunk 0 is
// fetched during the last chunk of the current one, so no tile pays the DMA round trip of its first
// chunk or a workgroup launch, and the 2 workgroups of a CU drift out of phase (one's epilogue
// stores under the other's MFMAs).  Needs an even chunk count (the operand-buffer parity restarts at
// every tile) and a slot count per XCD divisible by the channel blocks (launch_dma).  Experiments
// build only (PMU_DMA_PERS=1): bit-identical to the one-tile grid (tests/test_dma_pers_gpu.py) but
// SLOWER on every c5 shape — kbench --c5 fwd 4.92 vs 4.37 ms, dgrad 6.45 vs 4.73 (profiles/r05/pers):
// state carried across the tile loop spills 60-80 VGPRs, and a scratch reload in the chunk loop waits
// (in-order vmcnt) for the DMA issued before it, serialising the fetch pipeline.
template <bool DGRAD, bool ZB, int WN, int NWV, int EXP = 0, bool CS = false, bool XB = false, bool PERS = false>
__global__ __launch_bounds__(64 * NWV, 8 / NWV) void conv3x3_dma_kernel(DmaArgs a) {
  using G = DG<WN, NWV>;
  constexpr int FM = 4, FN = 2, BN = G::BN, WM = G::WM, TH = G::TH, NT = G::NT;
  // (PERS: the epilogue's reduction area apart from the stages, which hold the next tile's chunk 0)
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * G::STAGE + (PERS ? NT * 8 : 0)];
  // the wave index as a uniform (SGPR) value: the epilogue's row pointers derive from it
  const int tid = threadIdx.x, lane = tid & 63, wave = DGRAD ? tid >> 6 : __builtin_amdgcn_readfirstlane(tid >> 6);
  // (spatial tile, channel block), channel blocks fastest in XCD order: the channel blocks of one
  // tile share its halo image through their XCD's L2
  int cb, tcur, tend = 0, tstride = 0;
  if constexpr (PERS) {
    // slot s of XCD x (workgroups are dispatched round-robin over the 8 XCDs): channel block s % ncb,
    // tiles start + s / ncb, + nsl / ncb, ... of the XCD's contiguous share [start, tend)
    const int x = blockIdx.x & 7, s = blockIdx.x >> 3, nsl = gridDim.x >> 3;
    const int T = a.N * a.tiles_h * a.tiles_w, q = T >> 3, r = T & 7;
    const int start = x * q + (x < r ? x : r);
    cb = s % a.ncb;
    tend = start + q + (x < r ? 1 : 0);
    tstride = nsl / a.ncb;
    tcur = start + s / a.ncb;
    if (tcur >= tend) return;
  } else {
    const int lb = pmu_xcd_block(blockIdx.x, gridDim.x);
    cb = lb % a.ncb;
    tcur = lb / a.ncb;
  }
  const int j0 = cb * BN;
  int tsp, n, h0, w0;
  auto coords = [&](int t, int& tn, int& th0, int& tw0) {
    const int tw = t % a.tiles_w;
    t /= a.tiles_w;
    th0 = (t % a.tiles_h) * TH;
    tn = t / a.tiles_h;
    tw0 = tw * TW;
  };
  tsp = tcur;
  coords(tcur, n, h0, w0);
  PMU_DCHECK(n < a.N && j0 < a.NOUT, PMU_DBG_GRID);

  f32x16 acc[FM][FN];
  bf16x8 op[2][FM + FN];
  bool first = true;
  for (;;) {  // tiles (one unless PERS)
  // (PERS: the lane is opaque per tile, so every lane-derived address is formed inside the tile
  // instead of hoisted out of the tile loop and held through the epilogue: 100-200 VGPRs spilled)
  int tl = lane;
  if constexpr (PERS) asm volatile("" : "+v"(tl));
  // operand units of this thread (DMA round r: unit (r * 8 + wave) * 64 + lane): 32-bit byte offset
  // of chunk 0 and whether the unit is inside the image; units outside it are zero in both stages
  unsigned goff[G::NGA];
  unsigned gin = 0u;
  auto offsets = [&](int tn, int th0, int tw0) {
    gin = 0u;
#pragma unroll
    for (int r = 0; r < G::NGA; ++r) {
      const int u = (r * NWV + wave) * 64 + tl;
      const bool data = u < G::A_UNITS;
      const int hp = u >> 1, q = (u & 1) ^ ((hp >> 3) & 1);
      const int hr = hp / HW2, hc = hp - hr * HW2;
      const int h = th0 - 1 + hr, w = tw0 - 1 + hc;
      const bool in = data && h >= 0 && w >= 0 && h < a.H && w < a.W;
      // (32-bit: the operand is under 4 GB, launch_dma; every partial product is at most the offset)
      goff[r] = in ? ((((unsigned)tn * a.H + h) * a.W + w) * a.Cp + 8 * q) * 2u : 0u;
      PMU_DCHECK(!in || (((long long)tn * a.H + h) * a.W + w) < (long long)a.N * a.H * a.W, PMU_DBG_OPERAND);
      gin |= in ? (1u << r) : 0u;
    }
  };
  // zero the units outside the image in one stage (the DMA skips them); PERS: before each tile's
  // first two fetches, the stages' previous contents being another tile's
  auto zero_stage = [&](unsigned char* st) {
#pragma unroll
    for (int r = 0; r < G::NGA; ++r) {
      const int u = (r * NWV + wave) * 64 + tl;
      if (u < G::A_UNITS && !((gin >> r) & 1u)) *reinterpret_cast<uint4*>(st + 16 * u) = make_uint4(0u, 0u, 0u, 0u);
    }
  };
  offsets(n, h0, w0);
  const char* wsrc = reinterpret_cast<const char*>(a.wp) + (long long)cb * a.nch * G::B_UNITS * 16 + 16 * tl;

#define PMU_GLDS(S, D)                                                                                      \
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(S),                     \
                                   (__attribute__((address_space(3))) void*)(D), 16, 0, 0);
#define PMU_FETCH(CH, STG)                                                                                  \
  {                                                                                                        \
    PMU_DCHECK((CH) * BK + BK <= a.Cp, PMU_DBG_OPERAND);                                                   \
    const char* xa_ = reinterpret_cast<const char*>(a.x) + (CH) * BK * 2;                                  \
    unsigned char* st_ = (STG);                                                                            \
    _Pragma("unroll") for (int r = 0; r < G::NGA; ++r)                                                     \
      if ((gin >> r) & 1u) PMU_GLDS(xa_ + goff[r], st_ + (r * NWV + wave) * 1024)                         \
    const char* wb_ = wsrc + (long long)(CH) * G::B_UNITS * 16;                                            \
    _Pragma("unroll") for (int r = 0; r < G::NGB; ++r)                                                     \
      if ((r + 1) * NT <= G::B_UNITS || (r * NWV + wave) * 64 + tl < G::B_UNITS)                            \
        PMU_GLDS(wb_ + (r * NWV + wave) * 1024, st_ + G::A_BYTES + (r * NWV + wave) * 1024)               \
  }

  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int q = tl >> 5, li = tl & 31;
  const int hpb = 4 * wm * HW2 + li;           // halo pixel of fragment 0, tap (0, 0)
  int ub[FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) ub[fn] = G::A_BYTES + 16 * swz(wn * 64 + fn * 32 + li, q);

  if (!PERS || first) {
    if constexpr (PERS) {
      zero_stage(smem);
    } else {
      zero_stage(smem);
      zero_stage(smem + G::STAGE);
    }
    PMU_FETCH(0, smem)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }  // (PERS, later tiles: chunk 0 fetched, landed and past the barrier in the last tile's last chunk)
  // One operand set per tap in two register buffers; tap t+1's reads are issued during tap t's MFMAs,
  // and the next chunk's tap 0 during this chunk's tap 8: the chunk barrier (its DMA landed, every
  // wave done reading the stage the following fetch overwrites) sits between two taps' MFMA groups,
  // not between a barrier and the first LDS round trip of a chunk.  9 taps per chunk flip the buffer
  // parity every chunk, so chunks run in compile-time-parity pairs.
  auto load_tap = [&](const unsigned char* cur, int tap, bf16x8 (&o)[FM + FN]) {
    const int dy = tap / 3, dx = tap - 3 * (tap / 3);
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int hp = hpb + (fm + dy) * HW2 + dx;
      o[fm] = *reinterpret_cast<const bf16x8*>(cur + 16 * swz(hp, q));
    }
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) o[FM + fn] = *reinterpret_cast<const bf16x8*>(cur + ub[fn] + tap * (32 * BN));
  };
  // (PERS) the next tile of this slot: tnext, at (nn, nh0, nw0)
  int tnext = 0, nn = 0, nh0 = 0, nw0 = 0;
  bool has_next = false;
  if constexpr (PERS) {
    tnext = tcur + tstride;
    has_next = tnext < tend;
    if (has_next) coords(tnext, nn, nh0, nw0);
  }
  auto run_chunk = [&](int ch, auto par) {
    constexpr int P = decltype(par)::value;
    const unsigned char* cur = smem + (ch & 1) * G::STAGE;
    const unsigned char* nxt = smem + ((ch + 1) & 1) * G::STAGE;
    const bool more = ch + 1 < a.nch || has_next;
    if (ch + 1 < a.nch) {
      if (PERS && ch == 0) zero_stage(smem + G::STAGE);
      PMU_FETCH(ch + 1, smem + ((ch + 1) & 1) * G::STAGE)
    } else if (PERS && has_next) {  // the next tile's chunk 0 (into stage 0: nch is even)
      offsets(nn, nh0, nw0);
      zero_stage(smem);
      PMU_FETCH(0, smem)
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      // this tap's operands (read during the previous tap's MFMAs) have landed: wait for them BEFORE
      // the next reads are issued (left to the compiler, an lgkmcnt(0) after those reads drained them
      // too: an LDS round trip with the MFMA pipe idle every other tap)
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt / expcnt at their maxima
      __builtin_amdgcn_sched_barrier(0);
      if (tap + 1 < 9) {
        load_tap(cur, tap + 1, op[(tap + 1 + P) & 1]);
      } else if (more) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's share of chunk ch + 1 landed
        __builtin_amdgcn_s_barrier();                      // everyone's, and every read of chunk ch - 1 done
        __builtin_amdgcn_sched_barrier(0);
        // (PERS, last chunk: the next tile's tap 0 is read at that tile's start, not held through the
        // epilogue)
        if (!PERS || ch + 1 < a.nch) load_tap(nxt, 0, op[(9 + P) & 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          if constexpr (!(EXP & 2))
            acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(op[(tap + P) & 1][fm], op[(tap + P) & 1][FM + fn],
                                                                   acc[fm][fn], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  load_tap(smem, 0, op[0]);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  int ch = 0;
  for (; ch + 1 < a.nch; ch += 2) {
    run_chunk(ch, std::integral_constant<int, 0>{});
    run_chunk(ch + 1, std::integral_constant<int, 1>{});
  }
  if (!PERS && ch < a.nch) run_chunk(ch, std::integral_constant<int, 0>{});
  if constexpr (!PERS) __syncthreads();  // every wave's last reads are done before the epilogue reuses the stages

  const int elane = tl, ej0 = j0;
  const int eli = elane & 31;
  // epilogue: accumulator (fm, fn, r) = output pixel (tile row 4 wm + fm, column acc_row(r, elane)),
  // channel ej0 + 64 wn + 32 fn + (elane & 31); a 32-channel destination is uniform (split % 32 == 0).
  // [NWV waves][64][2] (non-PERS: in the stages, free now)
  float* red = reinterpret_cast<float*>(smem + (PERS ? 2 * G::STAGE : 0));
  float s1[FN], s2[FN];
  if constexpr (!DGRAD) {
    // Forward: values and BN sums formed unconditionally (masked), only the stores predicated.  With the
    // bias first consumed inside a per-output branch the compiler waited vmcnt(0) in every branch,
    // i.e. for all earlier stores of the epilogue (one store in flight at a time: 112 waits for 128
    // stores).  Store addresses: a uniform row base per (fm, fn) + a 32-bit column offset.
    bool jok[FN];
    float bv[FN], zov[FN];
  #pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      s1[fn] = 0.f;
      s2[fn] = 0.f;
      const int j = ej0 + wn * 64 + fn * 32 + eli;
      jok[fn] = j < a.NOUT;
      const int jc = jok[fn] ? j : a.NOUT - 1;
      bv[fn] = a.bias ? a.bias[jc] : 0.f;
      zov[fn] = (ZB && a.zoff) ? a.zoff[jc] : 0.f;
    }
    // (ZB = false, NOUT even) z as 8-byte channel pairs: lanes 2k, 2k+1 hold adjacent channels of the
    // same pixels r, r + 1; one xor-1 shuffle gives the even elane pixel r's pair and the odd elane pixel
    // r + 1's — half the store instructions (the bf16 ConvT forward gained 23% from the same change)
    const bool pairs = !ZB && (a.NOUT & 1) == 0;
    const int odd = elane & 1;
  #pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int h = h0 + 4 * wm + fm;
      const long long rowpix = ((long long)n * a.H + (h < a.H ? h : a.H - 1)) * a.W;
      float* drow = a.out0 + rowpix * a.NOUT;
      unsigned short* drowb = reinterpret_cast<unsigned short*>(a.out0) + rowpix * a.NOUT;
      if (pairs) {
  #pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int j = ej0 + wn * 64 + fn * 32 + eli;
  #pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const float v0 = acc[fm][fn][r] + bv[fn], v1 = acc[fm][fn][r + 1] + bv[fn];
            const bool ok0 = jok[fn] && h < a.H && w0 + acc_row(r, elane) < a.W;
            const bool ok1 = jok[fn] && h < a.H && w0 + acc_row(r + 1, elane) < a.W;
            const float m0 = ok0 ? v0 : 0.f, m1 = ok1 ? v1 : 0.f;
            s1[fn] += m0;
            s2[fn] = fmaf(m0, m0, s2[fn]);
            s1[fn] += m1;
            s2[fn] = fmaf(m1, m1, s2[fn]);
            const float recv = pmu_swap1(odd ? v0 : v1);
            const float2 pv = odd ? make_float2(recv, v1) : make_float2(v0, recv);
            const int w = w0 + acc_row(r + odd, elane);
            if (!(jok[fn] && h < a.H && w < a.W) || (EXP & 1)) continue;
            PMU_DCHECK(((long long)n * a.H + h) * a.W + w < (long long)a.N * a.H * a.W, PMU_DBG_OUTPUT);
            st_drop(drow + (unsigned)(w * a.NOUT + j - odd), pv);
          }
        }
        continue;
      }
  #pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int j = ej0 + wn * 64 + fn * 32 + eli;
  #pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int w = w0 + acc_row(r, elane);
          const bool ok = jok[fn] && h < a.H && w < a.W;
          float v = acc[fm][fn][r] + bv[fn];
          unsigned short vb = 0;
          if (ZB) {
            vb = bf16_bits(v - zov[fn]);
            v = pmu_bf16_f32(vb) + zov[fn];
          }
          const float m = ok ? v : 0.f;
          s1[fn] += m;
          s2[fn] = fmaf(m, m, s2[fn]);
          if (!ok || (EXP & 1)) continue;
          PMU_DCHECK(((long long)n * a.H + h) * a.W + w < (long long)a.N * a.H * a.W, PMU_DBG_OUTPUT);
          const unsigned oo = (unsigned)(w * a.NOUT + j);
          if (ZB) drowb[oo] = vb;
          else drow[oo] = v;
        }
      }
    }
  } else {
    // Input gradient: all stores first, then (a.bz) the producer's BN-backward sums from the still-live
    // accumulators and the z under them, a row at a time.  z loads interleaved with the stores made
    // every consumption of a z value wait for all earlier stores (vmcnt counts both, in order); the
    // straight-line masked form of the forward above spilled 18-140 VGPRs here.
    // (XB: each use rounds its accumulator, rb() below; rounding all 128 up front spilled 7 VGPRs)
    auto rb = [](float v) { return XB ? pmu_round_bf16(v) : v; };
    // (a.bz) z under the accumulators, a fragment row (fn, fm) of 16 values per lane at a time, the next
    // row's loads issued before this row's are consumed (one HBM round trip per wave instead of one per
    // row), the first row's before the dx stores (its consumption then waits for no store); clamped
    // addresses: every elane loads, masked values ignored
    float zt[2][16];
    auto zload = [&](int g, float (&z)[16]) __attribute__((always_inline)) {
      const int fn = g / FM, fm = g - (g / FM) * FM;
      const int j = ej0 + wn * 64 + fn * 32 + eli;
      const int jc = j < a.NOUT ? j : a.NOUT - 1;
      const int h = h0 + 4 * wm + fm;
      const long long row = ((long long)n * a.H + min(h, a.H - 1)) * a.W;
  #pragma unroll
      for (int r = 0; r < 16; ++r) {
        const unsigned zo = (unsigned)(min(w0 + acc_row(r, elane), a.W - 1) * a.NOUT);
        if constexpr (ZB) z[r] = pmu_bf16_f32((reinterpret_cast<const unsigned short*>(a.bz) + row * a.NOUT + jc)[zo]);
        else z[r] = (a.bz + row * a.NOUT + jc)[zo];
      }
    };
    const bool bnr = !CS && a.bz;
    float bsc[FN], bsh[FN], bmu[FN], bis[FN];  // the producer's BN coefficients of the lane's channels
    if (bnr) {
      zload(0, zt[0]);
  #pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int j = ej0 + wn * 64 + fn * 32 + eli;
        const int jc = j < a.NOUT ? j : a.NOUT - 1;
        bsc[fn] = a.bcoef[jc];
        bsh[fn] = a.bcoef[a.NOUT + jc];
        bmu[fn] = a.bmean[jc];
        bis[fn] = a.binv[jc];
      }
    }
  #pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      s1[fn] = 0.f;
      s2[fn] = 0.f;
      const int jb = ej0 + wn * 64 + fn * 32;
      const int j = jb + eli;
      const bool jok = j < a.NOUT;
      float* dstp;
      int ld;
      unsigned short* dstb = nullptr;  // (uniform per fragment)
      if (jb < a.split) {
        ld = a.split;
        if constexpr (XB) { dstp = nullptr; dstb = reinterpret_cast<unsigned short*>(a.out0) + j; }
        else dstp = a.out0 + j;
      } else {  // (out1 null: only the bf16 copy, pmu_conv3x3_dgrad_dma_x1b_sum)
        dstp = a.out1 ? a.out1 + (j - a.split) : nullptr;
        ld = a.NOUT - a.split;
        if (a.out1b) dstb = a.out1b + (j - a.split);
      }
  #pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const int h = h0 + 4 * wm + fm;
        // the fragment row's first pixel (rows past the image clamped, their stores masked): one 64-bit
        // row base per (fm, fn), 32-bit offsets within the row
        const long long rowpix = ((long long)n * a.H + (h < a.H ? h : a.H - 1)) * a.W;
        if (dstb) {
          // the bf16 copy as 4-byte channel pairs: lanes 2k, 2k+1 hold adjacent channels of the same
          // pixels r, r + 1; one xor-1 shuffle gives the even elane pixel r's pair and the odd elane pixel
          // r + 1's (half the store instructions of 2-byte stores; dstb is uniform per fragment, so the
          // whole wave runs the shuffles; channel pairs never straddle NOUT: NOUT - split % 8 == 0)
          const int odd = elane & 1;
  #pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const unsigned b0 = bf16_bits(acc[fm][fn][r]), b1 = bf16_bits(acc[fm][fn][r + 1]);
            const unsigned recv = pmu_swap1(odd ? b0 : b1);
            const unsigned pair = odd ? (recv | (b1 << 16)) : (b0 | (recv << 16));
            const int w = w0 + acc_row(r + odd, elane);
            if (!jok || h >= a.H || w >= a.W) continue;
            PMU_DCHECK(rowpix + w < (long long)a.N * a.H * a.W, PMU_DBG_OUTPUT);
            st_drop(dstb + rowpix * ld + (unsigned)(w * ld - odd), pair);
          }
        }
        // (only CS has a null out1, its dx1 the bf16 copy alone; XB's dx0 is the bf16 store above)
        if ((CS || XB) && !dstp) continue;
        if ((ld & 1) == 0) {  // (uniform) fp32 dx as 8-byte channel pairs, as the bf16 copy above
          const int odd = elane & 1;
  #pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const float v0 = rb(acc[fm][fn][r]), v1 = rb(acc[fm][fn][r + 1]);
            const float recv = pmu_swap1(odd ? v0 : v1);
            const float2 pv = odd ? make_float2(recv, v1) : make_float2(v0, recv);
            const int w = w0 + acc_row(r + odd, elane);
            if (!jok || h >= a.H || w >= a.W) continue;
            PMU_DCHECK(rowpix + w < (long long)a.N * a.H * a.W, PMU_DBG_OUTPUT);
            st_drop(dstp + rowpix * ld + (unsigned)(w * ld - odd), pv);
          }
          continue;
        }
  #pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int w = w0 + acc_row(r, elane);
          if (!jok || h >= a.H || w >= a.W) continue;
          PMU_DCHECK(rowpix + w < (long long)a.N * a.H * a.W, PMU_DBG_OUTPUT);
          dstp[rowpix * ld + (unsigned)(w * ld)] = rb(acc[fm][fn][r]);
        }
      }
    }
    if (bnr) {
  #pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const bool jok = ej0 + wn * 64 + fn * 32 + eli < a.NOUT;
  #pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const int g = fn * FM + fm;
          if (g + 1 < FN * FM) zload(g + 1, zt[(g + 1) & 1]);
          const float (&z)[16] = zt[g & 1];
          const int h = h0 + 4 * wm + fm;
  #pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int w = w0 + acc_row(r, elane);
            const bool ok = jok && h < a.H && w < a.W;
            const float gg = (ok && fmaf(z[r], bsc[fn], bsh[fn]) > 0.f) ? rb(acc[fm][fn][r]) : 0.f;
            s1[fn] += gg;
            s2[fn] = fmaf(gg, (z[r] - bmu[fn]) * bis[fn], s2[fn]);
          }
        }
      }
    } else if (CS) {  // per-tile column sums of dx (x1b_sum: the transposed conv's bias gradient)
  #pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const bool jok = ej0 + wn * 64 + fn * 32 + eli < a.NOUT;
  #pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
          const int h = h0 + 4 * wm + fm;
  #pragma unroll
          for (int r = 0; r < 16; ++r) {
            const bool ok = jok && h < a.H && w0 + acc_row(r, elane) < a.W;
            s1[fn] += ok ? rb(acc[fm][fn][r]) : 0.f;
          }
        }
      }
    }
  }
  if (a.part) {  // forward: BN partial sums of the output; input gradient: of the producer's BN backward
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      s1[fn] += __shfl_xor(s1[fn], 32, 64);
      s2[fn] += __shfl_xor(s2[fn], 32, 64);
      if (elane < 32) {
        red[(wave * 64 + fn * 32 + elane) * 2 + 0] = s1[fn];
        red[(wave * 64 + fn * 32 + elane) * 2 + 1] = s2[fn];
      }
    }
    if constexpr (PERS) {  // (__syncthreads' vmcnt(0) would wait for every store of the epilogue)
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
    } else {
      __syncthreads();
    }
    if (tid < BN) {  // channel tid = 64 wn + c: summed over the WM waves of column group wn, in order
      const int j = ej0 + tid, wnn = tid >> 6, c = tid & 63;
      if (j < a.NOUT) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int m = 0; m < WM; ++m) {
          t1 += red[((m * WN + wnn) * 64 + c) * 2 + 0];
          t2 += red[((m * WN + wnn) * 64 + c) * 2 + 1];
        }
        PMU_DCHECK(tsp < a.N * a.tiles_h * a.tiles_w, PMU_DBG_WORKSPACE);
        a.part[((long long)tsp * 2 + 0) * a.NOUT + j] = t1;
        a.part[((long long)tsp * 2 + 1) * a.NOUT + j] = t2;
      }
    }
  }
  if constexpr (!PERS) {
    break;
  } else {
    if (!has_next) break;
    tcur = tsp = tnext;
    n = nn;
    h0 = nh0;
    w0 = nw0;
    first = false;
  }
  }  // tiles
#undef PMU_FETCH
#undef PMU_GLDS
}

// Workgroup shape: 64 output channels x 512 pixels in 4 waves (two workgroups per CU) for <= 64
// output channels or a short reduction (K <= 128 channels: a few chunks per tile, the prologue and
// the output stores are a large share); else 128 channels x 512 pixels in 8 waves
struct Shape {
  int wn, nwv, th;
};
static Shape dma_shape(int NOUT, int KC) {
#ifdef PMU_EXPERIMENTS
  // PMU_DMA_TALL=1 (A/B): the 64-channel workgroups as 8 waves over 32 tile rows (1024 pixels, one
  // workgroup per CU: half the tiles, a 34-row halo per 32 output rows instead of 18 per 16)
  static const int tall = [] {
    const char* e = pmu_variant_env("PMU_DMA_TALL");
    return e ? atoi(e) : 0;
  }();
  if (tall && dma_bn(NOUT, KC) == 64) return {1, 8, 32};
#endif
  if (dma_bn(NOUT, KC) == 64) return {1, 4, 16};
  return {2, 8, 16};
}

// persistent tiles (PERS above; experiments build, PMU_DMA_PERS=1) when every slot gets two or more:
// the resident workgroups per CU follow from the LDS (78 KB for the 4-wave shape, 117 KB for the
// 8-wave one)
static long long dma_slots(const Shape& sh) { return (long long)pmu_num_cus() * (sh.nwv == 4 ? 2 : 1); }
static bool dma_pers(const Shape& sh, int nch, int ncb, long long blocks) {
  const char* pe = pmu_variant_env("PMU_DMA_PERS");
  const long long slots = dma_slots(sh);
  return pe && atoi(pe) != 0 && sh.th == 16 && nch % 2 == 0 && slots % 8 == 0 && (slots / 8) % ncb == 0 &&
         blocks >= 2 * slots;
}

// one kernel variant by workgroup shape and tile schedule (pers: `slots` resident workgroups)
template <bool D, bool Z, bool CSV, bool XBV>
static void launch_variant(const Shape& sh, bool pers, dim3 grid, unsigned slots, hipStream_t st, const DmaArgs& a) {
  const dim3 blk(64 * sh.nwv);
#ifdef PMU_EXPERIMENTS
  if constexpr (!Z) {
    if (pers) {
      if (sh.wn == 1) hipLaunchKernelGGL((conv3x3_dma_kernel<D, Z, 1, 4, 0, CSV, XBV, true>), dim3(slots), blk, 0, st, a);
      else hipLaunchKernelGGL((conv3x3_dma_kernel<D, Z, 2, 8, 0, CSV, XBV, true>), dim3(slots), blk, 0, st, a);
      return;
    }
  }
#else
  (void)pers;
  (void)slots;
#endif
  if (sh.wn == 1 && sh.nwv == 4) hipLaunchKernelGGL((conv3x3_dma_kernel<D, Z, 1, 4, 0, CSV, XBV>), grid, blk, 0, st, a);
#ifdef PMU_EXPERIMENTS
  else if (sh.wn == 1 && sh.nwv == 8) hipLaunchKernelGGL((conv3x3_dma_kernel<D, Z, 1, 8, 0, CSV, XBV>), grid, blk, 0, st, a);
#endif
  else hipLaunchKernelGGL((conv3x3_dma_kernel<D, Z, 2, 8, 0, CSV, XBV>), grid, blk, 0, st, a);
}

static int launch_dma(const unsigned short* x, int Cp, int N, int H, int W, const unsigned short* wp, const float* bias,
                      int NOUT, float* out0, float* out1, int split, float* part, bool dgrad, void* stream,
                      const float* bz = nullptr, const float* bcoef = nullptr, const float* bmean = nullptr,
                      const float* binv = nullptr, int zbf = 0, const float* zoff = nullptr,
                      unsigned short* out1b = nullptr, bool xb = false) {
  PMU_REQUIRE(x && wp && out0 && N > 0 && H > 0 && W >= 32 && Cp > 0 && Cp % BK == 0 && NOUT > 0);
  PMU_REQUIRE(!out1b || dgrad);
  // bf16 dx: its channel pairs never straddle the split or the end (4-byte pair stores)
  PMU_REQUIRE(!xb || (dgrad && zbf == 0 && NOUT % 8 == 0 && split % 8 == 0));
  PMU_REQUIRE(!dgrad || split == NOUT || (split % 32 == 0 && split < NOUT && (out1 || out1b)));
  const Shape sh = dma_shape(NOUT, Cp);
  const long long img_bytes = (long long)H * W * Cp * 2;
  if ((long long)N * img_bytes >= (1LL << 32)) {  // 32-bit DMA byte offsets: split over images
    const long long tiles = (long long)pmu_cdiv(W, TW) * pmu_cdiv(H, sh.th);
    return pmu_image_chunks(N, img_bytes, [&](int n0, int nn) {
      const long long px = (long long)n0 * H * W;
      // bf16 z (forward output / input-gradient bz): element offsets of 2-byte values
      float* o0 = (!dgrad && zbf == 1) ? reinterpret_cast<float*>(reinterpret_cast<unsigned short*>(out0) + px * NOUT)
                  : xb ? reinterpret_cast<float*>(reinterpret_cast<unsigned short*>(out0) + px * split)
                       : out0 + px * (dgrad ? split : NOUT);
      const float* bzc = !bz ? nullptr
                             : zbf == 1 ? reinterpret_cast<const float*>(reinterpret_cast<const unsigned short*>(bz) + px * NOUT)
                                   : bz + px * NOUT;
      return launch_dma(x + px * Cp, Cp, nn, H, W, wp, bias, NOUT, o0, out1 ? out1 + px * (NOUT - split) : nullptr,
                        split, part ? part + (long long)n0 * tiles * 2 * NOUT : nullptr, dgrad, stream, bzc, bcoef,
                        bmean, binv, zbf, zoff, out1b ? out1b + px * (NOUT - split) : nullptr, xb);
    });
  }
  DmaArgs a;
  a.x = x; a.wp = wp; a.bias = bias; a.out0 = out0; a.out1 = out1; a.out1b = out1b; a.part = part;
  a.N = N; a.H = H; a.W = W; a.Cp = Cp; a.NOUT = NOUT; a.split = dgrad ? split : NOUT;
  a.nch = Cp / BK;
  a.bz = bz; a.bcoef = bcoef; a.bmean = bmean; a.binv = binv;
  a.zbf = zbf;
  a.zoff = zoff;
  a.ncb = pmu_cdiv(NOUT, 64 * sh.wn);
  a.tiles_w = pmu_cdiv(W, TW);
  a.tiles_h = pmu_cdiv(H, sh.th);
  const long long blocks = (long long)a.tiles_w * a.tiles_h * N * a.ncb;
  PMU_REQUIRE(blocks < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)blocks), blk(64 * sh.nwv);
  const bool zb = zbf == 1;
  const long long slots = dma_slots(sh);
  const bool pers = !zb && dma_pers(sh, a.nch, a.ncb, blocks);
#ifdef PMU_EXPERIMENTS
  {
    const char* e = pmu_variant_env("PMU_DMA_EXP");
    const int x = e ? atoi(e) : 0;
    if (!dgrad && !zb && x >= 1 && x <= 3 && !(sh.wn == 1 && sh.nwv == 8)) {
      if (sh.wn == 1) {
        if (x == 1) hipLaunchKernelGGL((conv3x3_dma_kernel<false, false, 1, 4, 1>), grid, blk, 0, st, a);
        if (x == 2) hipLaunchKernelGGL((conv3x3_dma_kernel<false, false, 1, 4, 2>), grid, blk, 0, st, a);
        if (x == 3) hipLaunchKernelGGL((conv3x3_dma_kernel<false, false, 1, 4, 3>), grid, blk, 0, st, a);
      } else {
        if (x == 1) hipLaunchKernelGGL((conv3x3_dma_kernel<false, false, 2, 8, 1>), grid, blk, 0, st, a);
        if (x == 2) hipLaunchKernelGGL((conv3x3_dma_kernel<false, false, 2, 8, 2>), grid, blk, 0, st, a);
        if (x == 3) hipLaunchKernelGGL((conv3x3_dma_kernel<false, false, 2, 8, 3>), grid, blk, 0, st, a);
      }
      PMU_CHECK_LAUNCH();
      return PMU_OK;
    }
  }
#endif
  const unsigned ns = (unsigned)slots;
  if (dgrad && part && !bz) {  // column sums (pmu_conv3x3_dgrad_dma_x1b_sum)
    if (xb) launch_variant<true, false, true, true>(sh, pers, grid, ns, st, a);
    else launch_variant<true, false, true, false>(sh, pers, grid, ns, st, a);
  } else if (dgrad && xb) {  // bf16 dx (the *_dxb entries)
    launch_variant<true, false, false, true>(sh, pers, grid, ns, st, a);
  }
#ifdef PMU_EXPERIMENTS
  else if (dgrad && zb) launch_variant<true, true, false, false>(sh, false, grid, ns, st, a);
  else if (zb) launch_variant<false, true, false, false>(sh, false, grid, ns, st, a);
#else
  else if (zb) return PMU_ERR_ARG;  // bf16-stored z: experiments build only
#endif
  else if (dgrad) launch_variant<true, false, false, false>(sh, pers, grid, ns, st, a);
  else launch_variant<false, false, false, false>(sh, pers, grid, ns, st, a);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

}  // namespace

extern "C" int pmu_conv3x3_dma_ok(int H, int W, int Cp, int NOUT, int split) {
  return W >= 32 && H >= 1 && Cp % BK == 0 && NOUT > 0 && (split == NOUT || split % 32 == 0);
}

#ifdef PMU_EXPERIMENTS
extern "C" int pmu_conv3x3_dma_persistent(int N, int H, int W, int NOUT, int Cp) {
  if (N <= 0 || H <= 0 || W < 32 || Cp <= 0 || Cp % BK || NOUT <= 0) return 0;
  const Shape sh = dma_shape(NOUT, Cp);
  const int ncb = pmu_cdiv(NOUT, 64 * sh.wn);
  const long long img_bytes = (long long)H * W * Cp * 2;
  // (an operand over 4 GB runs per image group: its first group's grid decides, as launch_dma does)
  long long n = N;
  if (n * img_bytes >= (1LL << 32)) n = std::max(1LL, ((1LL << 32) - 1) / img_bytes);
  const long long blocks = (long long)pmu_cdiv(W, TW) * pmu_cdiv(H, sh.th) * n * ncb;
  return dma_pers(sh, Cp / BK, ncb, blocks) ? 1 : 0;
}
#endif

extern "C" int pmu_conv3x3_tiles_dma(int N, int H, int W, int Cout, int Cp) {
  return N * pmu_cdiv(H, dma_shape(Cout, Cp).th) * pmu_cdiv(W, TW);
}

extern "C" size_t pmu_conv3x3_packed_size_dma(int Cout, int Cin, int dgrad) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  const int BN = dma_bn(NOUT, KC);
  return (size_t)pmu_cdiv(NOUT, BN) * pmu_cdiv(KC, BK) * 9 * 2 * BN * 8 * sizeof(unsigned short);
}

extern "C" int pmu_conv3x3_pack_dma(const float* w, int Cout, int Cin, int dgrad, unsigned short* wp, void* stream) {
  PMU_REQUIRE(w && wp && Cout > 0 && Cin > 0);
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  const long long total = (long long)(pmu_conv3x3_packed_size_dma(Cout, Cin, dgrad) / sizeof(unsigned short));
  long long g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(pack_dma_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, dgrad,
                     dma_bn(NOUT, KC), wp);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_conv3x3_fwd_dma(const unsigned short* xt, int Cp, int N, int H, int W, const unsigned short* wp,
                                   const float* bias, int Cout, float* z, float* part, void* stream) {
  return launch_dma(xt, Cp, N, H, W, wp, bias, Cout, z, nullptr, Cout, part, false, stream);
}

extern "C" int pmu_conv3x3_dgrad_dma(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                                     int Cin, int Csplit, float* dx0, float* dx1, void* stream) {
  return launch_dma(dzt, Cp, N, H, W, wp, nullptr, Cin, dx0, dx1, Csplit, nullptr, true, stream);
}

// The concat split input gradient with a bf16 copy of its second part (the transposed conv's bf16
// input gradient operand, which pmu_frame_to_bf16 would otherwise make from dx1 in another pass).
extern "C" int pmu_conv3x3_dgrad_dma_x1b(const unsigned short* dzt, int Cp, int N, int H, int W,
                                         const unsigned short* wp, int Cin, int Csplit, float* dx0, float* dx1,
                                         unsigned short* dx1b, void* stream) {
  PMU_REQUIRE(dx1 && dx1b && Csplit < Cin && (Cin - Csplit) % 8 == 0);
  return launch_dma(dzt, Cp, N, H, W, wp, nullptr, Cin, dx0, dx1, Csplit, nullptr, true, stream, nullptr, nullptr,
                    nullptr, nullptr, 0, nullptr, dx1b);
}

// As pmu_conv3x3_dgrad_dma_x1b with dx1 kept only in bf16, plus per-tile column sums of dx in
// part[tile][0][Cin] (part[tile][1][*] = 0; tiles = pmu_conv3x3_tiles_dma(N, H, W, Cin, Cp)): the
// transposed conv's bias gradient is the sum over tiles of channels [Csplit, Cin)
// (pmu_convT2x2_dbias_rows), so its fp32 du is neither written nor re-read.
extern "C" int pmu_conv3x3_dgrad_dma_x1b_sum(const unsigned short* dzt, int Cp, int N, int H, int W,
                                             const unsigned short* wp, int Cin, int Csplit, float* dx0,
                                             unsigned short* dx1b, float* part, void* stream) {
  PMU_REQUIRE(dx1b && part && Csplit < Cin && (Cin - Csplit) % 8 == 0);
  return launch_dma(dzt, Cp, N, H, W, wp, nullptr, Cin, dx0, nullptr, Csplit, part, true, stream, nullptr, nullptr,
                    nullptr, nullptr, 0, nullptr, dx1b);
}

// As pmu_conv3x3_dgrad_wino4_bnr (part rows = pmu_conv3x3_tiles_dma(N, H, W, Cin, Cp)).
extern "C" int pmu_conv3x3_dgrad_dma_bnr(const unsigned short* dzt, int Cp, int N, int H, int W, const unsigned short* wp,
                                         int Cin, float* dx, const float* z, const float* coef, const float* mean,
                                         const float* invstd, float* part, void* stream) {
  PMU_REQUIRE(z && coef && mean && invstd && part);
  return launch_dma(dzt, Cp, N, H, W, wp, nullptr, Cin, dx, nullptr, Cin, part, true, stream, z, coef, mean, invstd);
}

// bf16 dx (XB above): as the entries without the _dxb suffix, with dx / dx0 stored as bf16 (RNE, the
// dtype torch.autocast's conv backward returns) and every other output formed from the rounded values.
// Cin % 8 == 0, Csplit % 8 == 0.
extern "C" int pmu_conv3x3_dgrad_dma_dxb(const unsigned short* dzt, int Cp, int N, int H, int W,
                                         const unsigned short* wp, int Cin, int Csplit, unsigned short* dx0,
                                         float* dx1, void* stream) {
  return launch_dma(dzt, Cp, N, H, W, wp, nullptr, Cin, reinterpret_cast<float*>(dx0), dx1, Csplit, nullptr, true,
                    stream, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, true);
}

extern "C" int pmu_conv3x3_dgrad_dma_x1b_dxb(const unsigned short* dzt, int Cp, int N, int H, int W,
                                             const unsigned short* wp, int Cin, int Csplit, unsigned short* dx0,
                                             float* dx1, unsigned short* dx1b, void* stream) {
  PMU_REQUIRE(dx1 && dx1b && Csplit < Cin && (Cin - Csplit) % 8 == 0);
  return launch_dma(dzt, Cp, N, H, W, wp, nullptr, Cin, reinterpret_cast<float*>(dx0), dx1, Csplit, nullptr, true,
                    stream, nullptr, nullptr, nullptr, nullptr, 0, nullptr, dx1b, true);
}

extern "C" int pmu_conv3x3_dgrad_dma_x1b_sum_dxb(const unsigned short* dzt, int Cp, int N, int H, int W,
                                                 const unsigned short* wp, int Cin, int Csplit, unsigned short* dx0,
                                                 unsigned short* dx1b, float* part, void* stream) {
  PMU_REQUIRE(dx1b && part && Csplit < Cin && (Cin - Csplit) % 8 == 0);
  return launch_dma(dzt, Cp, N, H, W, wp, nullptr, Cin, reinterpret_cast<float*>(dx0), nullptr, Csplit, part, true,
                    stream, nullptr, nullptr, nullptr, nullptr, 0, nullptr, dx1b, true);
}

extern "C" int pmu_conv3x3_dgrad_dma_bnr_dxb(const unsigned short* dzt, int Cp, int N, int H, int W,
                                             const unsigned short* wp, int Cin, unsigned short* dx, const float* z,
                                             const float* coef, const float* mean, const float* invstd, float* part,
                                             void* stream) {
  PMU_REQUIRE(z && coef && mean && invstd && part);
  return launch_dma(dzt, Cp, N, H, W, wp, nullptr, Cin, reinterpret_cast<float*>(dx), nullptr, Cin, part, true, stream,
                    z, coef, mean, invstd, 0, nullptr, nullptr, true);
}

#ifdef PMU_EXPERIMENTS
// (experiments build only: bf16 z breaks the c5 Dice contract)
// bf16 storage of z (config c5's autocast dtype), centred on zoff (the BN running mean; null: 0): the
// forward stores bf16(z - zoff) (RNE) with the BN partial sums of stored + zoff; the input gradient's
// BN-backward partials read such a z with the centred coefficients (shift + zoff*scale, mean - zoff).
extern "C" int pmu_conv3x3_fwd_dma_zb(const unsigned short* xt, int Cp, int N, int H, int W, const unsigned short* wp,
                                      const float* bias, int Cout, unsigned short* z, const float* zoff, float* part,
                                      void* stream) {
  return launch_dma(xt, Cp, N, H, W, wp, bias, Cout, reinterpret_cast<float*>(z), nullptr, Cout, part, false, stream,
                    nullptr, nullptr, nullptr, nullptr, 1, zoff);
}

extern "C" int pmu_conv3x3_dgrad_dma_bnr_zb(const unsigned short* dzt, int Cp, int N, int H, int W,
                                            const unsigned short* wp, int Cin, float* dx, const unsigned short* z,
                                            const float* coef, const float* mean, const float* invstd, float* part,
                                            void* stream) {
  PMU_REQUIRE(z && coef && mean && invstd && part);
  return launch_dma(dzt, Cp, N, H, W, wp, nullptr, Cin, dx, nullptr, Cin, part, true, stream,
                    reinterpret_cast<const float*>(z), coef, mean, invstd, 1);
}

#endif  // PMU_EXPERIMENTS

static int pack_dma_grid(int Cout, int Cin, int dgrad) {
  const long long total = (long long)(pmu_conv3x3_packed_size_dma(Cout, Cin, dgrad) / sizeof(unsigned short));
  const long long g = (total + 255) / 256;
  return (int)(g > 4096 ? 4096 : g);
}

extern "C" int pmu_conv3x3_pack_dma_blocks(int Cout, int Cin, int dgrad) { return pack_dma_grid(Cout, Cin, dgrad); }

extern "C" int pmu_conv3x3_pack_dma_multi(const pmu_pack_job* jobs, int njobs, int blocks, int dgrad, void* stream) {
  PMU_REQUIRE(jobs && njobs > 0 && blocks > 0);
  hipLaunchKernelGGL(pack_dma_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, jobs, njobs, dgrad);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

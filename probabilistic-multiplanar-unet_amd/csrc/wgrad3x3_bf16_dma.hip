// Weight gradient of the 3x3 / pad 1 convolution on bf16 MFMA with both operands staged by LDS-DMA
// (config c5: autograd of nn.Conv2d w.r.t. its weight, PMU/model/unet/unet_parts.py:15,18, under
// torch.autocast(bfloat16): bf16 operands, fp32 sums, fp32 dw).
//
//   dw[co][ci][kh][kw] = sum_{n,y,x} dzt[n,y,x,co] * xt[n, y+kh-1, x+kw-1, ci]
//
// GEMM per wave: one 32-co x 32-ci fragment pair and ALL nine taps (9 accumulators of
// v_mfma_f32_32x32x16_bf16, 144 registers); K = pixels, 16 per k-step = one 16-pixel row segment of a
// vertical strip of the image.  A workgroup walks its strips down, row by row:
//   * the dz row (A) of step y serves all nine taps;
//   * the three activation rows y-1, y, y+1 (B, per kw a 16-pixel window of an 18-pixel halo row)
//     are kept in registers and rotate: each step reads ONE new halo row (y+1), the rows for kh = 0, 1
//     come from the two previous steps.
// Per step and wave: 2 + 6 ds_read_b64_tr_b16 for 9 MFMAs (the register-staged kernel in
// wgrad3x3_bf16.hip: 10 for 6).
//
// Staging: a ring of NS LDS stages filled by global_load_lds (16 B per lane, no staging registers, no
// ds_write); a stage holds three consecutive steps (dz rows y..y+2, halo rows y+1..y+3) of every strip
// lane of the workgroup; one barrier per two stages (54 MFMAs per wave; a ring of 5: kbench over the
// c5 shapes 4.21 vs 4.29 ms with one barrier per stage and a ring of 4, profiles/r05/wgrad_pair).  Units outside the image, the
// channels or the segment read zeros through the buffer descriptors' range check, so every wave issues
// the same number of DMA instructions per stage and the ring waits are counted (s_waitcnt vmcnt(N)) with
// the next NS-2 stages in flight.  LDS rows are unit permutations, not padded rows (LDS-DMA writes 1 KiB contiguous per
// wave-instruction): 16-B unit u of pixel p sits at u ^ sw(p), chosen so the four pixel rows a 32-lane
// group of a transposed read touches fall in four distinct 16-bank quarters (conflict-free).
//
// K split: the image is cut into segments (n, 16-wide strip, 3m consecutive rows); a segment starts
// with a prologue stage (halo rows y0-1, y0 into the rotation registers).  Workgroup = (co block, ci
// block, split); its WS strip lanes each walk SPB segments in lockstep; split-K slabs
// ws[split*WS + lane][tap][co][ci], reduced in a fixed order (pmu_splitk_reduce9_kernel).
#include <type_traits>

#include "pmu_stage.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));


constexpr int SW = 16;  // strip width (pixels per k-step)

// WCOF x WCIF x WS = 8 waves: co fragments x ci fragments x strip lanes; TPS step triplets per stage
template <int WCOF, int WCIF, int WS, int TPS>
struct WG {
  static_assert(WCOF * WCIF * WS == 8, "8 waves");
  static constexpr int NT = 512;
  static constexpr int ARU = 4 * WCOF, XRU = 4 * WCIF;      // 16-B units per pixel row
  // LDS rows of whole wave-instructions (64 units): every DMA instruction moves units of ONE image row,
  // so its row, and whether that row lies in the image, are uniform (SGPR) per instruction and stage; the
  // halo row's 18 pixels are padded (144 -> 192 units at 8 per pixel, 288 -> 320 at 16; the pad reads
  // zeros and is never read back)
  static constexpr int A_ROW = SW * ARU, X_ROW = ((SW + 2) * XRU + 63) / 64 * 64;
  static_assert(A_ROW % 64 == 0, "dz rows of whole wave-instructions");
  // a strip lane's three dz rows and three halo rows, each region rounded up to whole wave-instructions
  // (64 units), so every DMA instruction moves one kind of one strip lane: its kind, lane and row step
  // are uniform per (instruction, wave)
  static constexpr int RPS = 3 * TPS;                        // rows per stage
  static constexpr int A_LANE = (RPS * A_ROW + 63) / 64 * 64, X_LANE = (RPS * X_ROW + 63) / 64 * 64;
  static constexpr int A_UNITS = WS * A_LANE, X_UNITS = WS * X_LANE;
  static constexpr int NI = (A_UNITS + X_UNITS + NT - 1) / NT;  // DMA instructions per wave per stage
  static constexpr int STAGE = NI * NT * 16;                      // bytes
  // PAIR: one barrier per two stages (a ring of 5: the barrier at an even stage s waits for s and
  // s + 1 and refills the two slots s - 2, s - 1 free by then); else one per stage, a ring of 4 / 3
  static constexpr bool PAIR = 5 * STAGE <= 160 * 1024;
  static constexpr int NS = PAIR ? 5 : (4 * STAGE <= 160 * 1024) ? 4 : 3;
  static_assert(NS * STAGE <= 160 * 1024, "LDS");
};

// unit permutation of a pixel row of F 32-channel fragments (see top)
template <int F>
__device__ __forceinline__ int wgd_sw(int p) {
  return F == 1 ? 0 : F == 2 ? 4 * ((p >> 1) & 1) : 4 * (p & 3);
}

struct WgdArgs {
  const unsigned short* dzt;  // [N][H][W][Cop]
  const unsigned short* xt;   // [N][H][W][Cip]
  float* ws;
  int N, H, W, Cout, Cin, Cop, Cip;
  unsigned bytesA, bytesX;    // dzt / xt bytes (< 2^31: buffer-descriptor range, see the kernel)
  int strips_w, nseg_strip, m, spb, nsplit, nseg;  // segments: 3m rows; spb per lane; nseg in all
};

template <int OFF>
__device__ __forceinline__ s16x4 wgd_tr(unsigned addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int N>
__device__ __forceinline__ void wgd_wait_lgkm() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt");
  __builtin_amdgcn_s_waitcnt(0xC07F | (N << 8));
}
__device__ __forceinline__ bf16x8 wgd_frag(s16x4 lo, s16x4 hi) {
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int N>
__device__ __forceinline__ void wgd_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  // gfx9 s_waitcnt: vmcnt[3:0] bits 3:0, vmcnt[5:4] bits 15:14; expcnt / lgkmcnt at their maxima
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

// EXP (timing experiments, experiments build, PMU_WGD_EXP; wrong results on purpose): 1 = no DMA at all
// (the stage bookkeeping and barriers kept), 2 = every DMA through the zero-record descriptor (addresses
// formed, nothing fetched), 3 = the DMA as shipped without the stage barrier
template <int WCOF, int WCIF, int WS, int TPS, int EXP = 0>
__global__ __launch_bounds__(512, 2) void wgrad3x3_bf16_dma_kernel(WgdArgs a) {
  using G = WG<WCOF, WCIF, WS, TPS>;
  constexpr int RPS = G::RPS;
  constexpr int NS = G::NS, NI = G::NI;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ncb = pmu_cdiv_dev(a.Cout, 32 * WCOF), nib = pmu_cdiv_dev(a.Cin, 32 * WCIF);
  // (channel block, split) in XCD order, channel blocks fastest: the blocks of one split walk the same
  // pixels in step on one XCD, whose L2 then serves each row to all of them
  const int nblk = ncb * nib;
  const int lbk = pmu_xcd_block(blockIdx.x, gridDim.x);
  const int blk = lbk % nblk, split = lbk / nblk;
  const int co0 = (blk % ncb) * 32 * WCOF, ci0 = (blk / ncb) * 32 * WCIF;
  PMU_DCHECK(split < a.nsplit, PMU_DBG_GRID);
  // wave -> (co fragment, ci fragment, strip lane)
  const int wco = wave % WCOF, wci = (wave / WCOF) % WCIF, wsl = wave / (WCOF * WCIF);

  // segment (lane sl, k-th of the block) -> image n, strip column c0, first row y0 (none: k past the
  // block's segments or the launch's — y0 beyond the image, so every unit reads zeros)
  auto seg_of = [&](int k, int sl, int& n, int& c0, int& y0) __attribute__((always_inline)) {
    const int s = (split * a.spb + k) * WS + sl;
    if (k >= a.spb || s >= a.nseg) { n = 0; c0 = 0; y0 = a.H + 1; return; }
    const int ys = s % a.nseg_strip;
    const int st = s / a.nseg_strip;
    c0 = (st % a.strips_w) * SW;
    n = st / a.strips_w;
    y0 = ys * RPS * a.m;
  };
  // DMA of stage index s (segment k = s / (m+1), step t = s % (m+1)) into ring slot s % NS.  Stage t = 0:
  // halo rows y0-1, y0, y0+1 (the prologue; dz rows unread); t >= 1: dz rows Y..Y+2 and halo rows
  // Y+1..Y+3, Y = y0 + 3(t-1).  Lane unit U = (i * 8 + wave) * 64 + lane of the stage.  Stages are issued
  // in order, so a cursor (dk, dt, slot) replaces the divisions.
  // Sources are buffer loads to LDS (buffer_load_dwordx4 ... lds) through SGPR descriptors: the byte
  // address = descriptor base + soffset (SGPR: the instruction's image row, uniform) + voffset (VGPR: the
  // lane's pixel and channel within the row, fixed per segment).  Units outside the image or the
  // channels read zeros through the range check: a lane outside the row carries voffset 0x80000000
  // (>= every descriptor's size, tensors < 2^31 bytes: pmu_conv3x3_wgrad_dma_ok), an instruction whose
  // row is outside the image (or whose segment is none) goes through the zero-record descriptor.  A
  // stage's DMA issue is SALU work plus the DMA instructions — no per-lane address arithmetic (the 64-bit
  // global_load_lds addresses and their in-image selects were ~10 VALU per DMA: kbench over the c5 shapes
  // 3.53 ms with them formed but unused vs 3.07 without, EXP 4 / 2 of round 6).
  // (every descriptor input and soffset is made provably wave-uniform with readfirstlane: otherwise hipcc
  // wraps each buffer op in a waterfall loop, and a select between whole descriptors went through scratch)
  const unsigned rbA = 2u * a.W * a.Cop, rbX = 2u * a.W * a.Cip;   // bytes per image row
  // per instruction i, for the current segment: yr = n*H + y (image row index) and yl = y (row in the
  // image, range check) at stage t = 1 — uniform; vo = the lane's byte offset within the row
  int yr[NI], yl[NI];
  unsigned vo[NI];
  auto seg_setup = [&](int k) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int w = i * 8 + wave;                    // wave-instruction index of the stage (uniform)
      const bool isA = w * 64 < G::A_UNITS;
      const int sl = isA ? (w * 64) / G::A_LANE : (w * 64 - G::A_UNITS) / G::X_LANE;
      const int ROW = isA ? G::A_ROW : G::X_ROW;
      const int rb = isA ? w * 64 - sl * G::A_LANE : w * 64 - G::A_UNITS - sl * G::X_LANE;  // (uniform)
      const int j = rb / ROW;                                                              // (uniform)
      const int pu = rb - j * ROW + lane;
      const int px = isA ? pu / G::ARU : pu / G::XRU;
      const int u = isA ? ((pu % G::ARU) ^ wgd_sw<WCOF>(px)) : ((pu % G::XRU) ^ wgd_sw<WCIF>(px));
      int n, c0, y0;
      seg_of(k, sl < WS ? sl : 0, n, c0, y0);
      const int x = isA ? c0 + px : c0 - 1 + px;
      const int c = 8 * u + (isA ? co0 : ci0);
      const int Cp = isA ? a.Cop : a.Cip;
      const bool in = px < (isA ? SW : SW + 2) && x >= 0 && x < a.W && c < Cp;
      vo[i] = in ? (unsigned)(x * Cp + c) * 2u : 0x80000000u;
      const bool rowok = sl < WS && j < RPS;
      const int y1 = y0 + j + (isA ? 0 : 1);         // the instruction's row at stage t = 1
      yl[i] = __builtin_amdgcn_readfirstlane(rowok ? y1 : -(1 << 28));  // (outside: never inside [0, H))
      yr[i] = __builtin_amdgcn_readfirstlane(n * a.H + y1);
    }
  };
  int dk = 0, dt = 0, dslot = 0;
  seg_setup(0);
  auto issue = [&]() __attribute__((always_inline)) {
    unsigned char* stg = smem + dslot * G::STAGE;
    // rows relative to stage t = 1: dz RPS(t-1) (none at t = 0); halo RPS(t-1), at t = 0 -2 (y0-1, ..)
    const int dyA = RPS * (dt - 1), dyX = dt == 0 ? -2 : RPS * (dt - 1);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if constexpr (EXP == 1) continue;
      const bool isA = (i * 8 + wave) * 64 < G::A_UNITS;   // (uniform)
      const int dy = isA ? dyA : dyX;
      const bool ok = EXP != 2 && (unsigned)(yl[i] + dy) < (unsigned)a.H && (!isA || dt > 0);
      const int soff = __builtin_amdgcn_readfirstlane((int)((unsigned)(yr[i] + dy) * (isA ? rbA : rbX)));
      const int nrec = __builtin_amdgcn_readfirstlane(ok ? (int)(isA ? a.bytesA : a.bytesX) : 0);
#if defined(__HIP_DEVICE_COMPILE__)  // (the descriptor type and builtins exist for the device pass only; a
                                     // template body using them in the host pass lost the kernel's stub)
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<unsigned short*>(isA ? a.dzt : a.xt), 0, nrec, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(stg + (i * 8 + wave) * 1024),
                                               16, vo[i], soff, 0, 0);
#else
      (void)soff; (void)nrec; (void)stg;
#endif
    }
    dslot = dslot + 1 == NS ? 0 : dslot + 1;
    if (++dt > a.m) {   // (uniform) the next stage starts a new segment
      dt = 0;
      seg_setup(++dk);
    }
  };

  f32x16 acc[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // transposed-read lane roles: half h takes pixels 8h..8h+7 of the 16-pixel step, group g the column
  // block 16g of the fragment, lane 4q+p supplies pixel row 4t+q (t = 0, 1: the two reads) and columns
  // 4p..4p+3 (byte 8 (p & 1) of 16-B unit 2g + (p >> 1) of the fragment).  Byte offsets within a stage,
  // per lane (row j of the stage adds the immediate offset j * row bytes).
  const int h = lane >> 5, g = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
  const int ua = wco * 4 + 2 * g + (p >> 1), ux = wci * 4 + 2 * g + (p >> 1), hb = 8 * (p & 1);
  const int aoff = wsl * G::A_LANE, xoff = G::A_UNITS + wsl * G::X_LANE;
  unsigned ra[2], rx[3][2];
#pragma unroll
  for (int t2 = 0; t2 < 2; ++t2) {
    const int pa = 8 * h + 4 * t2 + q;
    ra[t2] = 16u * (aoff + pa * G::ARU + (ua ^ wgd_sw<WCOF>(pa))) + hb;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int px = pa + kw;
      rx[kw][t2] = 16u * (xoff + px * G::XRU + (ux ^ wgd_sw<WCIF>(px))) + hb;
    }
  }
  const unsigned sbase = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)(smem);
  // The LDS reads are inline asm: through the ds_read_tr intrinsic the compiler cannot tell them from
  // the pending LDS-DMA writes and put an s_waitcnt vmcnt(0) before every stage's reads (the whole ring
  // drained each stage).  Their results are waited for by hand (wgd_wait_lgkm) behind a scheduling
  // barrier, so no MFMA moves above its wait.
  auto rd_a = [&](unsigned st, auto J) __attribute__((always_inline)) {
    constexpr int OFF = decltype(J)::value * G::A_ROW * 16;
    return wgd_frag(wgd_tr<OFF>(st + ra[0]), wgd_tr<OFF>(st + ra[1]));
  };
  auto rd_x = [&](unsigned st, auto J, bf16x8 (&o)[3]) __attribute__((always_inline)) {
    constexpr int OFF = decltype(J)::value * G::X_ROW * 16;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) o[kw] = wgd_frag(wgd_tr<OFF>(st + rx[kw][0]), wgd_tr<OFF>(st + rx[kw][1]));
  };
  auto mm = [&](const bf16x8& af, const bf16x8 (&k0)[3], const bf16x8 (&k1)[3],
                const bf16x8 (&k2)[3]) __attribute__((always_inline)) {
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      acc[0][kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, k0[kw], acc[0][kw], 0, 0, 0);
      acc[1][kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, k1[kw], acc[1][kw], 0, 0, 0);
      acc[2][kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, k2[kw], acc[2][kw], 0, 0, 0);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  // prologue: the first NS-1 stages in flight (stages past the end read the zero page or other segments
  // into slots nobody reads, so every wave issues NI DMAs per stage index and the counted waits hold)
#pragma unroll
  for (int s = 0; s < NS - (G::PAIR ? 2 : 1); ++s) issue();
  // (a segment's prologue and its triplets as nested loops: as the two arms of one per-stage branch,
  // the merged rotation registers spilled 150+ VGPRs)
  int rslot = 0;   // ring slot of stage s (s % NS)
  int sg = 0;      // stage index s (PAIR: its parity)
  auto begin_stage = [&]() __attribute__((always_inline)) {
    if constexpr (G::PAIR) {
      // even s: stages s and s + 1 landed (this wave's DMAs: all but the NS-4 younger stages'), then
      // every wave's, and every read of stage s - 1 done; then stages s + NS - 2, s + NS - 1 into the
      // slots of s - 2, s - 1.  Odd s: nothing (covered by the even barrier before it)
      if ((sg & 1) == 0) {
        wgd_wait_vm<(NS - 4) * NI>();
        if constexpr (EXP != 3) __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        issue();
        issue();
        __builtin_amdgcn_sched_barrier(0);
      }
      ++sg;
    } else {
      // stage s landed (this wave's DMAs: all but the NS-2 younger stages'), then every wave's, and every
      // read of stage s-1 — whose slot the next DMA overwrites — is done (its MFMAs consumed them)
      wgd_wait_vm<(NS - 2) * NI>();
      if constexpr (EXP != 3) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      issue();   // stage s + NS - 1, into the slot stage s - 1 used
      __builtin_amdgcn_sched_barrier(0);
    }
    const unsigned st = sbase + (unsigned)(rslot * G::STAGE);
    rslot = rslot + 1 == NS ? 0 : rslot + 1;
    return st;
  };
  // halo rows y-1, y of the next step (per kw) in two register sets that alternate per triplet: a
  // triplet reads (P0, P1) and leaves its last two halo rows in (Q0, Q1), the next triplet the other
  // way round — no rotation copies (12 bf16x8 moves per triplet, ~0.9 VALU per MFMA, in a kernel that
  // is instruction-issue-bound)
  bf16x8 B0[3], B1[3], C0[3], C1[3];
  // triplet TT of a stage: steps on its rows 3TT .. 3TT+2 (read during the previous step's MFMAs)
  auto triplet = [&](unsigned st, auto TT, const bf16x8 (&P0)[3], const bf16x8 (&P1)[3], bf16x8 (&Q0)[3],
                     bf16x8 (&Q1)[3]) __attribute__((always_inline)) {
    constexpr int T0 = 3 * decltype(TT)::value;
    bf16x8 x0[3];
    const bf16x8 a0 = rd_a(st, std::integral_constant<int, T0>{});
    rd_x(st, std::integral_constant<int, T0>{}, x0);
    const bf16x8 a1 = rd_a(st, std::integral_constant<int, T0 + 1>{});
    rd_x(st, std::integral_constant<int, T0 + 1>{}, Q0);
    wgd_wait_lgkm<8>();  // step y's 8 reads
    __builtin_amdgcn_sched_barrier(0);
    mm(a0, P0, P1, x0);
    __builtin_amdgcn_sched_barrier(0);
    const bf16x8 a2 = rd_a(st, std::integral_constant<int, T0 + 2>{});
    rd_x(st, std::integral_constant<int, T0 + 2>{}, Q1);
    wgd_wait_lgkm<8>();  // step y+1's
    __builtin_amdgcn_sched_barrier(0);
    mm(a1, P1, x0, Q0);
    __builtin_amdgcn_sched_barrier(0);
    wgd_wait_lgkm<0>();
    __builtin_amdgcn_sched_barrier(0);
    mm(a2, x0, Q0, Q1);
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int k = 0; k < a.spb; ++k) {
    {  // prologue of a segment: halo rows y0-1, y0
      const unsigned st = begin_stage();
      rd_x(st, I0{}, B0);
      rd_x(st, I1{}, B1);
      wgd_wait_lgkm<0>();
      __builtin_amdgcn_sched_barrier(0);
    }
    // TPS triplets per stage of steps y, y+1, y+2 (new halo rows y+1, y+2, y+3); the register sets
    // alternate B -> C -> B, so stages run in pairs (TPS = 1) and a segment's odd last one alone (its
    // C rows are not read: the next segment's prologue reloads B)
    if constexpr (TPS == 2) {
      for (int t = 1; t <= a.m; ++t) {
        const unsigned st = begin_stage();
        triplet(st, I0{}, B0, B1, C0, C1);
        triplet(st, I1{}, C0, C1, B0, B1);
      }
    } else {
      int t = 1;
      for (; t + 1 <= a.m; t += 2) {
        unsigned st = begin_stage();
        triplet(st, I0{}, B0, B1, C0, C1);
        st = begin_stage();
        triplet(st, I0{}, C0, C1, B0, B1);
      }
      if (t <= a.m) triplet(begin_stage(), I0{}, B0, B1, C0, C1);
    }
  }
  wgd_wait_vm<0>();  // (the tail stages' DMAs: nothing of them is read; drained before the wave exits)

  // slab write: ws[split * WS + lane][tap][co][ci]; accumulator rows = co, columns = ci (lanes)
  const int sp = split * WS + wsl;
  const int ci = ci0 + wci * 32 + (lane & 31);
  if (ci < a.Cin) {
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int tap = kh * 3 + kw;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = co0 + wco * 32 + acc_row(r, lane);
          PMU_DCHECK(sp < a.nsplit * WS, PMU_DBG_WORKSPACE);
          if (co < a.Cout) a.ws[(((long long)sp * 9 + tap) * a.Cout + co) * a.Cin + ci] = acc[kh][kw][r];
        }
      }
  }
}

struct WgdGeo {
  int wcof, wcif, ws, tps, nsplit, m, spb, nseg_strip, strips_w, nseg;
};

// Workgroup shape by channel counts, then the K split: about one workgroup per CU in all (256), whole
// strips per segment when there are enough of them, else strips cut into equal row segments.
static WgdGeo wgd_geometry(int N, int H, int W, int Cin, int Cout) {
  WgdGeo g;
  if (Cout <= 64 && Cin <= 64) { g.wcof = 2; g.wcif = 2; g.ws = 2; }
  else if (Cout <= 64) { g.wcof = 2; g.wcif = 4; g.ws = 1; }
  else { g.wcof = 4; g.wcif = 2; g.ws = 1; }
  // one step triplet per stage (TPS = 2, half the barriers per MFMA, spilled 26 VGPRs at its 160 KB ring)
  g.tps = 1;
  const int rps = 3 * g.tps;
  const int nb = pmu_cdiv(Cout, 32 * g.wcof) * pmu_cdiv(Cin, 32 * g.wcif);
  g.nsplit = 256 / nb;
  if (g.nsplit < 1) g.nsplit = 1;
  g.strips_w = pmu_cdiv(W, SW);
  const long long strips = (long long)N * g.strips_w;
  const long long lanes = (long long)g.nsplit * g.ws;
  g.nseg_strip = strips >= lanes ? 1 : (int)((lanes + strips - 1) / strips);
  if (g.nseg_strip > pmu_cdiv(H, rps)) g.nseg_strip = pmu_cdiv(H, rps);
  g.m = pmu_cdiv(pmu_cdiv(H, g.nseg_strip), rps);
  g.nseg_strip = pmu_cdiv(H, rps * g.m);
  g.nseg = (int)(strips * g.nseg_strip);
  if ((long long)g.nsplit * g.ws > g.nseg) g.nsplit = pmu_cdiv(g.nseg, g.ws);
  g.spb = pmu_cdiv(g.nseg, g.nsplit * g.ws);
  g.nsplit = pmu_cdiv(g.nseg, g.spb * g.ws);  // (no workgroup without a segment)
  return g;
}

}  // namespace

// Shapes the LDS-DMA weight gradient takes (the engine's default for bf16 maps at least 16 wide).
extern "C" int pmu_conv3x3_wgrad_dma_ok(int N, int H, int W, int Cin, int Cout) {
  const long long px = (long long)N * H * W;
  // (buffer descriptors: each operand below 2^31 bytes, so offsets and the out-of-range marker fit)
  return N > 0 && H > 0 && W >= SW && Cin > 0 && Cout > 0 && 2 * px * ((Cin + 7) & ~7) < (1LL << 31) &&
         2 * px * ((Cout + 7) & ~7) < (1LL << 31);
}

extern "C" size_t pmu_conv3x3_wgrad_ws_bf16_dma(int N, int H, int W, int Cin, int Cout) {
  const WgdGeo g = wgd_geometry(N, H, W, Cin, Cout);
  return (size_t)g.nsplit * g.ws * 9 * Cout * Cin * sizeof(float);
}

// dw[Cout][Cin][3][3] from dzt [N][H][W][pad8(Cout)] and xt [N][H][W][pad8(Cin)] (bf16), as
// pmu_conv3x3_wgrad_bf16; ws holds pmu_conv3x3_wgrad_ws_bf16_dma() bytes.
extern "C" int pmu_conv3x3_wgrad_bf16_dma(const unsigned short* dzt, const unsigned short* xt, int N, int H, int W,
                                          int Cout, int Cin, float* dw, float* ws, size_t ws_bytes, void* stream) {
  PMU_REQUIRE(dzt && xt && dw && ws && pmu_conv3x3_wgrad_dma_ok(N, H, W, Cin, Cout));
  const WgdGeo g = wgd_geometry(N, H, W, Cin, Cout);
  PMU_REQUIRE(ws_bytes >= (size_t)g.nsplit * g.ws * 9 * Cout * Cin * sizeof(float));
  WgdArgs a;
  a.dzt = dzt; a.xt = xt; a.ws = ws;
  a.N = N; a.H = H; a.W = W; a.Cout = Cout; a.Cin = Cin;
  a.Cop = (Cout + 7) & ~7; a.Cip = (Cin + 7) & ~7;
  a.bytesA = (unsigned)(2LL * N * H * W * a.Cop);
  a.bytesX = (unsigned)(2LL * N * H * W * a.Cip);
  a.strips_w = g.strips_w; a.nseg_strip = g.nseg_strip; a.m = g.m; a.spb = g.spb; a.nsplit = g.nsplit;
  a.nseg = g.nseg;
  const int nb = pmu_cdiv(Cout, 32 * g.wcof) * pmu_cdiv(Cin, 32 * g.wcif);
  const dim3 grid((unsigned)(nb * g.nsplit)), blk(512);
  hipStream_t st = (hipStream_t)stream;
#ifdef PMU_EXPERIMENTS
  static const int exp_v = [] {
    const char* e = pmu_variant_env("PMU_WGD_EXP");
    return e ? atoi(e) : 0;
  }();
  if (exp_v >= 1 && exp_v <= 3) {
#define PMU_WGD_LAUNCH(E)                                                                                   \
    if (g.ws == 2) hipLaunchKernelGGL((wgrad3x3_bf16_dma_kernel<2, 2, 2, 1, E>), grid, blk, 0, st, a);      \
    else if (g.wcof == 2) hipLaunchKernelGGL((wgrad3x3_bf16_dma_kernel<2, 4, 1, 1, E>), grid, blk, 0, st, a); \
    else hipLaunchKernelGGL((wgrad3x3_bf16_dma_kernel<4, 2, 1, 1, E>), grid, blk, 0, st, a);
    if (exp_v == 1) { PMU_WGD_LAUNCH(1) } else if (exp_v == 2) { PMU_WGD_LAUNCH(2) } else { PMU_WGD_LAUNCH(3) }
#undef PMU_WGD_LAUNCH
  } else
#endif
  if (g.ws == 2) hipLaunchKernelGGL((wgrad3x3_bf16_dma_kernel<2, 2, 2, 1>), grid, blk, 0, st, a);
  else if (g.wcof == 2) hipLaunchKernelGGL((wgrad3x3_bf16_dma_kernel<2, 4, 1, 1>), grid, blk, 0, st, a);
  else hipLaunchKernelGGL((wgrad3x3_bf16_dma_kernel<4, 2, 1, 1>), grid, blk, 0, st, a);
  PMU_CHECK_LAUNCH();
  const long long E = 9LL * Cout * Cin;
  hipLaunchKernelGGL(pmu_splitk_reduce9_kernel, dim3((unsigned)pmu_cdiv(E, 64)), dim3(256), 0, st, (const float*)ws,
                     g.nsplit * g.ws, (long long)Cout * Cin, dw);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

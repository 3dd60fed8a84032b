// Rolling-depth implicit-GEMM Conv3d 3x3x3 on MFMA for 16-bit channels-last
// views (gfx950): the forward of DUF's dense-unit convs nn.Conv3d(F, 32, 3,
// padding=(p, 1, 1)) (duf_net.py:203,214) and, with a mode-1 packed weight and
// depth padding 2 - p, their input gradient (loss.backward(),
// base_trainer.py:128).
//
// Why not conv_fast (conv_fast_impl.h), whose stage is (kd tap, 32 input
// channels): every input slice was staged three times (once per kd tap), the
// 9-tap weight slice once per stage, and a two-slot ring kept one stage
// (~1 us of MFMA work) in flight.  PMC on the DUF F->32 conv: MFMA pipes 27 %
// busy, 35 % of wave time parked at the per-stage vmcnt(0) + barrier, 1.6x the
// algorithmic HBM bytes.  Here:
//  * A stage is (input depth slice di, 16 input channels).  The slice is
//    staged ONCE and feeds all three kd taps: the workgroup keeps three
//    accumulator banks acc[kd] = output depth di + pd - kd and rotates them
//    when the walk moves to the next slice (the bank that leaves holds a
//    finished output depth, which is stored).  Bytes per MFMA: 3.3 B/KFLOP
//    (was 6.0).
//  * The stage's weight slab (27 taps x 32 output channels x 16 input
//    channels) rides in the same slot; taps of a kd with no output depth in
//    the tile are fetched from the zero page (no L2 traffic).
//  * Three 48 KB slots: the DMA of stage g+2 is issued while stage g
//    computes, so two stages (~3 us) of lookahead cover the HBM latency.
//  * 32-byte LDS rows, the two 16-byte pieces of a row XOR-swizzled by bit 3
//    of the row's halo column (A) or output channel (B): every ds_read_b128
//    lane group touches 16 distinct (row mod 8, piece) pairs = all 64 banks.
//  * Every DMA wave-instruction count is the same for every wave and stage
//    (47 real 1 KB pieces + 1 junk piece per slot, 6 per wave), so each wait
//    is a compile-time vmcnt that leaves exactly the next stage in flight.
//
// Tile: 8 waves x 2 rows x 32 columns x 32 output channels x a run of output
// depths [z0, z1) of one sample.  MFMA v_mfma_f32_32x32x16_{bf16,f16},
// operands "weights x voxels" (a lane's accumulator column is one voxel).
//
// Sub-pixel forms (2-D only, SP = 1 / 2): DRF's strided Conv2d /
// ConvTranspose2d(k, s, p) projections run as 3x3 convs on the low-res grid
// over a shuffle-s input (SP 1) or output (SP 2) view (drf_net.py:70-102,
// vsrk_subpixel_conv_weight).  Each sub-pixel phase of the shuffled operand
// meets only a 2 x 2 (k = 2s) window of the 3 x 3 taps; the other taps' weights
// are structurally zero and their MFMAs are skipped (a per-phase tap mask:
// 4 of 9 taps at k = 8, s = 4, p = 2).
#include <cstdlib>
#include "conv_common.h"

#ifndef ROLL_NT
#define ROLL_NT 0  // A/B: non-temporal output stores in the transposed epilogue
#endif
typedef uint32_t roll_u32x4 __attribute__((ext_vector_type(4)));
typedef int roll_v4i __attribute__((ext_vector_type(4)));
// Raw buffer resource over [base, base + 2 GiB) (wave-uniform base): offsets
// at or beyond 0x7FFFFFF0 read as zero and drop stores -- the register-
// transposed epilogue's out-of-range voxels without branches
typedef __amdgpu_buffer_rsrc_t RRsrc;
constexpr uint32_t ROLL_OOB = 0x80000000u;
__device__ __forceinline__ RRsrc roll_rsrc(const void* base) {
  const uint64_t b = (uint64_t)base;
  const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, 0, 0x7FFFFFF0, 0x00020000);
}
__device__ __forceinline__ uint4 roll_bload16(RRsrc r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
// SWAP (2-D forms without a prefetched operand): the flush transposes the
// accumulators in registers (epilogue_sw) instead of parking them in LDS;
// measured on the EDSR 64 -> 64 body (profiles/r6_roll_defer_ab.txt, nodefer):
// plain forward -13 %, data gradient -7 %, ReLU forward -5 %, while the
// prefetched-operand 2-D forms and the 3-D forms lost 3-4 % with it and keep
// the LDS park (0 builds the park everywhere)
#ifndef ROLL_SWAP
#define ROLL_SWAP 1
#endif
// PREF2D: the residual / mask operand of a 2-D tile prefetched into
// registers during the slice's last stages (0: loaded in the flush, which
// then takes the SWAP form)
#ifndef ROLL_PREF2D
#define ROLL_PREF2D 1
#endif
// SWAP_PREF: the register-transposed flush also for the prefetched residual /
// mask forms (their prefetch then in the swap lanes' layout)
// PFEARLY: the 2-D operand prefetch issued this many stages earlier than the
// slice's third-to-last (A/B knob)
#ifndef ROLL_PFEARLY
#define ROLL_PFEARLY 0
#endif
#ifndef ROLL_SWAP_PREF
#define ROLL_SWAP_PREF 0
#endif

namespace {
using namespace vsrk_conv;

// waves per workgroup and output rows per wave (A/B builds: -DROLL_RNW=4
// -DROLL_RMS=4 keeps the 16-row tile with one wave per SIMD)
#ifndef ROLL_RNW
#define ROLL_RNW 8
#endif
#ifndef ROLL_RMS
#define ROLL_RMS 2
#endif
constexpr int RNW = ROLL_RNW;              // waves (2 per SIMD)
constexpr int RMS = ROLL_RMS;              // output rows per wave
constexpr int RFTH = RNW * RMS;            // 16 tile rows
constexpr int RHW = TW + 2;                // 34 halo columns
constexpr int RHROWS = (RFTH + 2) * RHW;   // 612 halo voxels
constexpr int RCH = 16;                    // input channels per stage
constexpr int RNAI = (RHROWS + 31) / 32;   // 20 A pieces (32 voxels x 32 B each)
constexpr int RNA = (RNAI + RNW - 1) / RNW;  // 3: A pieces per wave (q < 3)
constexpr int RNSLOT = 3;
// Ablation builds for measurements only (tools/build_exp_multi.sh ... -DROLL_ABL=n;
// results are wrong): 1 no MFMAs, 2 no DMA pieces, 4 no epilogue, 8 no
// fragment reads, 16 no stage barrier
#ifndef ROLL_ABL
#define ROLL_ABL 0
#endif
// ROLL_LEAN (default 1): cheaper DMA piece issue -- M0 set without saving /
// restoring it (nothing else in these kernels uses M0: checked in the ISA),
// the zero page address held in a VGPR pair instead of re-materialised per
// piece, the A / B role of a piece resolved at compile time where every wave
// agrees, and every stage issues its pieces unconditionally (zero-page pieces
// past the end of the walk) so each wait is one compile-time vmcnt with no
// branch; 0 builds the previous form for A/B
#ifndef ROLL_LEAN
#define ROLL_LEAN 1
#endif
// (The epilogue operand prefetch is a plain compiler-visible load; round 4's
// inline-asm variant, whose destination registers the compiler could re-use
// before the data landed, is gone.)


// Geometry of the two forms.  KD = 3, NT = 1: Conv3d 3x3x3, one 32-channel
// output block, three accumulator banks (output depths).  KD = 1, NT = 2:
// Conv 3x3 over depth-1 slices (a Conv2d on a D = 1 view), two 32-channel
// output blocks sharing every A fragment (the 64-channel EDSR body convs).
// B piece p = tap * NT + nt holds (tap, output block nt): 32 channels x 32 B.
// WR (resident weights): the whole weight image of the output block -- every
// input chunk's B pieces, nchunk x NB KB -- is loaded into LDS once (per
// workgroup, or when the walk enters another output block) instead of riding
// in every stage's slot.  The LDS-DMA issue of a piece costs ~60-185 cycles
// beside MFMAs (MI355X_MICROARCH.md) and the ablations of this kernel showed
// the DMA pieces at about a third of its time: a stage then brings the 20 A
// pieces only (EDSR body 64 -> 64: 38 -> 20 pieces; DUF data gradient
// 32 -> F: 47 -> 20).
template <int KD, int NT, int WR = 0>
struct RollGeo {
  static_assert((KD == 3 && NT == 1) || (KD == 1 && (NT == 2 || NT == 1)),
                "rolling conv forms: 3x3x3 / 32, 3x3 / 64 or (folded depth) 3x3 / 32");
  static constexpr int NB = 9 * KD * NT;           // B pieces: 27 / 18
  static constexpr int NI = WR ? RNAI : RNAI + NB;  // 47 / 38 (WR: 20)
  static constexpr int NQ = (NI + RNW - 1) / RNW;  // pieces per wave and stage: 6 / 5 (WR: 3)
  // 48 KB / 40 KB: A | B | junk pieces.  WR: 24 KB (2-D: the transposed
  // epilogue parks a row in two halves, 2 KB per wave) or 32 KB (3-D: room
  // for the one-pass 4 KB park; the fourth piece per wave is never loaded)
  static constexpr int SLOT = (WR && KD == 3 && NQ < 4 ? 4 : NQ) * RNW * 1024;
  static constexpr int PPW = SLOT / (RNW * 1024);  // slot pieces per wave (the epilogue's park scratch)
  static constexpr int NACC = KD * NT;             // accumulator sets: banks (KD 3) or blocks (KD 1)
  static constexpr int NG = 3 * NACC;              // compute groups (kw, set): 9 / 6
  // groups 0 .. NDG-1 issue the next-but-one stage's pieces, PPG each; the
  // rest carry the late prologue (8 waves: one piece per group)
  static constexpr int NDG = NQ < NG - 1 ? NQ : NG - 1;
  static constexpr int PPG = (NQ + NDG - 1) / NDG;
  static constexpr int NTG = NG - NDG;             // groups that carry the late prologue: 3 / 1
  static constexpr int TPG = (RNA + NTG - 1) / NTG;
  static_assert(NTG >= 1, "a group must be left for the late prologue");
};

// Epilogue forms (compile time): out = fma(acc, out_scale, bias*out_scale)
// [relu | prelu] [* (mask > 0)] [+ residual] [+ out]
// RE_PMASK: the PReLU backward of the output's consumer fused in (mask = the
// PReLU's forward output at y's element offsets; * a where it is <= 0) with
// per-lane partials of the slope gradient (drf_net.py:56-106 PReLUs);
// with RE_ACC the mask applies to the accumulated sum (out + conv: the
// consumer's gradient is complete only after this last contribution)
// RE_BNRED (3-D form): the reduce half of the BN+ReLU backward whose dz this
// data gradient is (duf_net.py:198-203: bn2 before conv2) fused into the
// epilogue: per tile and wave, (sum dy', sum dy' xhat) of its 32 channels
// with dy' = out * (bnx * scale + shift > 0), xhat = (bnx - mean) * invstd
// (the per-tile partials hold sum dy' (bnx - mean); the final kernel scales
// by invstd)
enum { RE_RES = 1, RE_MASK = 2, RE_ACC = 4, RE_RELU = 8, RE_PRELU = 16, RE_PMASK = 32, RE_BNRED = 64 };
// sub-pixel operand (2-D forms): none, input view, output view.  SP_FOLD:
// the depth-folded form of a Conv3d 3x3x3 with one output depth from three
// input slices (DUF's last unit, padding (0, 1, 1), duf_net.py:214): a 3x3
// conv over the (kd, channel) chunks of the three slices -- chunk i reads
// slice kd = sptap[i] at element offset spoff[i] and the weights of depth tap
// kd (fold_wstride elements apart in the packed [kd][kh][kw][co][ci] image)
enum { SP_NONE = 0, SP_X = 1, SP_Y = 2, SP_FOLD = 3 };
constexpr int RMAXSUB = 64;  // chunk / block table entries (1024 logical channels)

// Division by a launch constant d (dividends < 2^31): q = (x * mul) >> p with
// p = 31 + ceil(log2 d), mul = ceil(2^p / d).
struct RDiv {
  uint32_t d, mul, p;
};
RDiv make_rdiv(int d) {
  int l = 0;
  while ((1u << l) < (uint32_t)d) ++l;
  const uint32_t p = 31 + l;
  return RDiv{(uint32_t)d, (uint32_t)(((1ull << p) + (uint64_t)d - 1) / (uint64_t)d), p};
}
__device__ __forceinline__ int rdiv(int x, const RDiv& f) { return (int)(((uint64_t)(uint32_t)x * f.mul) >> f.p); }

// 32-bit element strides (the host checks that every offset fits)
struct RView {
  char* ptr;
  int d, h, w;
  int sn, sd, sh, sw;
};

struct RollArgs {
  RView x, y, res, msk;
  const void* w;
  const float* bias;
  const float* pro_scale;
  const float* pro_shift;
  int cin, cout, cin_pad, cout_pad;
  int pd, ph, pw;
  int prologue;
  int bias_r;  // > 1: bias in torch pixel-shuffle order (a y_shuffle output of perm-packed weights)
  float out_scale;
  int dzc, nchunk, ntiles;
  RDiv ntn, nzc, tiles_w, tiles_h;
  // sub-pixel forms: per input chunk (SP_X) / 32-channel output block (SP_Y),
  // the element offset of its channels inside the shuffled operand (phase
  // row / column + physical channel) and its tap mask (bit kh*3 + kw)
  const float* act_param;
  int prio;  // A/B knob (VSRK_ROLL_PRIO=1): s_setprio 1 for waves 4-7 (MI355X_MICROARCH.md, two waves per SIMD)
  // SP_FOLD: input chunks per depth tap, element stride of a depth tap in the
  // packed weights, logical channels of the prologue tables (3 x cin; their
  // constants repeat every cin)
  int fold_nc, fold_wstride, fold_tab, fold_cin;
  const float* mask_slope;  // RE_PMASK: the PReLU slope a (device scalar)
  double* slope_part;       // RE_PMASK: [block][wave] partials of the slope gradient
  // RE_BNRED: the BN input (y's geometry and strides), its per-channel
  // constants and the [tile][wave][2 halves][16 sum + 16 sum-xhat] slab
  const char* bnx;
  const float *bn_sc, *bn_sh, *bn_mu, *bn_is;
  float* red_ws;
  int spoff[RMAXSUB];
  uint16_t sptap[RMAXSUB];
};

__device__ __attribute__((aligned(256))) uint4 g_roll_zero[16];
#ifdef ROLL_STAMP
// Diagnostic builds only (tools/roll_stamps.py): s_memtime stamps of waves 0
// and 4 (one SIMD) of workgroups 0-15, kept in VGPR lanes during the walk
// (no memory operation inside the pipeline) and stored at exit: per step
// [after the stage wait, after the barrier, after the flush, after compute]
#ifndef ROLL_STAMP_SKIP
#define ROLL_STAMP_SKIP 8
#endif
__device__ unsigned g_roll_stamp[16 * 2 * 128];
#endif

template <int N>
__device__ __forceinline__ void roll_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int KD, int NT, int PRO, int EM, int SP, typename H, int WR>
__global__ __launch_bounds__(RNW * 64, RNW / 4) void conv_roll_kernel(RollArgs a) {
  static_assert(SP == SP_NONE || KD == 1, "sub-pixel views: 2-D form only");
  static_assert(!WR || SP == SP_NONE, "resident weights: plain views only");
  using G = RollGeo<KD, NT, WR>;
  constexpr int RNQ = G::NQ, RSLOT = G::SLOT, NACC = G::NACC;
  // the transposed epilogue parks a row in two halves (2 KB of scratch per
  // wave) where the slot is too small for one 4 KB park (WR)
#ifdef ROLL_PARK2
  constexpr bool PARK2 = ROLL_PARK2 || G::PPW < 4;
#else
  constexpr bool PARK2 = G::PPW < 4;
#endif
  // the residual / mask operand of a 2-D tile is loaded into registers during
  // its last stage (one extra operand, no accumulate)
  // (3-D: the BN input of RE_BNRED, read by the flush of the slice's finished depth)
  constexpr bool PREF = (ROLL_PREF2D && KD == 1 && ((EM & RE_RES) != 0) != ((EM & RE_MASK) != 0) && !(EM & RE_ACC)) ||
                        (KD == 3 && (EM & RE_BNRED) != 0);
  constexpr bool SWAP = ROLL_SWAP && KD == 1 && (!PREF || ROLL_SWAP_PREF);
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (a.prio && wave >= 4) __builtin_amdgcn_s_setprio(1);
  char* wres = lds + RNSLOT * RSLOT;  // WR: [chunk][B piece] 1 KB pieces of the resident output block
  float* lbias = reinterpret_cast<float*>(wres + (WR ? a.nchunk * G::NB * 1024 : 0));  // [cout_pad] bias * out_scale
  // (SP_FOLD: the tables span the fold's 3 x cin logical channels)
  const int tabc = SP == SP_FOLD ? a.fold_tab : a.cin_pad;
  float* lsc = lbias + a.cout_pad;                                // [cin_pad] prologue scale / shift
  float* lsh = lsc + tabc;
  if constexpr (PRO) {
    if constexpr (SP == SP_FOLD) {
      for (int i = tid; i < tabc; i += RNW * 64) {
        const int c = i % a.fold_cin;
        const bool aff = (a.prologue & VSRK_PRO_AFFINE) != 0;
        lsc[i] = aff ? a.pro_scale[c] : 1.f;
        lsh[i] = aff ? a.pro_shift[c] : 0.f;
      }
    } else {
      stage_prologue(lsc, lsh, a.prologue, a.pro_scale, a.pro_shift, a.cin, a.cin_pad, tid, RNW * 64);
    }
  }
  for (int i = tid; i < a.cout_pad; i += RNW * 64) {
    float b = 0.f;
    if (a.bias && i < a.cout) {
      int cb = i;
      if (a.bias_r > 1) {  // view order (sub, c') -> torch order c' * r * r + sub
        const int rr = a.bias_r * a.bias_r, cp = a.cout / rr;
        const int sub = cb / cp;
        cb = (cb - sub * cp) * rr + sub;
      }
      b = a.bias[cb];
    }
    lbias[i] = b * a.out_scale;
  }
  // RE_BNRED: [4][cout_pad] BN constants after the prologue tables
  float* lbn = lbias + a.cout_pad + 2 * tabc;
  if constexpr ((EM & RE_BNRED) != 0) {
    for (int i = tid; i < a.cout_pad; i += RNW * 64) {
      const bool ok = i < a.cout;
      lbn[i] = ok ? a.bn_sc[i] : 0.f;
      lbn[a.cout_pad + i] = ok ? a.bn_sh[i] : 0.f;
      lbn[2 * a.cout_pad + i] = ok ? a.bn_mu[i] : 0.f;
      lbn[3 * a.cout_pad + i] = ok ? a.bn_is[i] : 0.f;
    }
  }
  // RE_BNRED: this lane's partials of its 8-channel column (lane & 3) of the
  // transposed epilogue
  constexpr int NRS = (EM & RE_BNRED) ? 8 : 1;
  float rs1[NRS], rs2[NRS];
#pragma unroll
  for (int i = 0; i < NRS; ++i) rs1[i] = rs2[i] = 0.f;

  // ---- per-lane DMA roles, fixed for the launch ----
  // piece j = wave + RNW*q fills slot bytes [j KB, j+1 KB); lane l writes 16
  // bytes at j KB + 16 l.  A (j < RNAI): halo voxel v = 32 j + l/2 (row
  // hh = v / 34, column ww = v % 34), position l & 1 holds the logical piece
  // p = (l & 1) ^ bit 3 of ww (8 channels).  B (j < NI): piece j - RNAI =
  // (tap, output block), output channel l/2, piece p = (l & 1) ^ bit 3 of
  // the channel.  qa: the wave's A pieces (bit q); qkd[kd]: its B pieces of
  // taps of depth kd.
  int rel[RNQ], hwv[RNQ];
  // qa in closed form: pieces q < RNAI / RNW are A pieces on every wave, so
  // the compiler resolves their role at compile time
  const unsigned qa = ((1u << (RNAI / RNW)) - 1) | (wave < RNAI % RNW ? 1u << (RNAI / RNW) : 0u);
  unsigned qkd0 = 0, qkd1 = 0, qkd2 = 0;
#pragma unroll
  for (int q = 0; q < RNQ; ++q) {
    const int j = wave + RNW * q;
    rel[q] = 0;
    hwv[q] = -1;
    if (j < RNAI) {
      const int v = 32 * j + (lane >> 1);
      const int hh = v / RHW, ww = v - (v / RHW) * RHW;
      const int p = (lane & 1) ^ ((ww >> 3) & 1);
      rel[q] = hh * a.x.sh + ww * a.x.sw + 8 * p;
      hwv[q] = v < RHROWS ? ((hh << 8) | ww) : -1;
    } else if (j < G::NI) {
      const int co = lane >> 1;
      const int p = (lane & 1) ^ ((co >> 3) & 1);
      const int tap = (j - RNAI) / NT, nt = (j - RNAI) % NT;
      rel[q] = (tap * a.cout_pad + nt * 32 + co) * a.cin_pad + 8 * p;
      const int kd = tap / 9;
      if (kd == 0) qkd0 |= 1u << q;
      else if (kd == 1) qkd1 |= 1u << q;
      else qkd2 |= 1u << q;
    }
  }
  // ds_read bases (bytes within a slot): A fragment (kw, halo row hr) at
  // abase[kw] + hr * 34 * 32; B fragment (tap, block) at RNAI KB + piece KB + bbase.
  uint32_t abase[3];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
    abase[kw] = (uint32_t)((wave * RMS * RHW + kw + r) * 32 + 16 * (hf ^ (((kw + r) >> 3) & 1)));
  // (WR: the B pieces of the stage's chunk in the resident image, same piece layout)
  const uint32_t bbase = (uint32_t)((WR ? 0 : RNAI * 1024) + r * 32 + 16 * (hf ^ ((r >> 3) & 1)));

  // ---- tiles of this workgroup (XCD group x owns a contiguous range) ----
  const int G_ = gridDim.x;
  const int xg = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int gx = (G_ >> 3) + (xg < (G_ & 7) ? 1 : 0);
  const int cx = xg * (G_ >> 3) + min(xg, G_ & 7);
  const int t_lo = (int)((int64_t)a.ntiles * cx / G_);
  const int t_hi = (int)((int64_t)a.ntiles * (cx + gx) / G_);

  // A tile as the walks need it.  Order: output-channel tile fastest (they
  // share the input), then the depth run, columns, rows, sample.
  struct RTile {
    int t;  // tile index
    int h0, w0, n0, z0, z1, di_lo, nsl, nb;
    int xo;  // element offset of halo origin (nb, di = 0, h0 - ph, w0 - pw) in x
    int yo;  // element offset of (nb, dz = 0, h0, w0, n0) in y
  };
  auto decode = [&](int t) __attribute__((always_inline)) {
    RTile tl;
    tl.t = t;
    int u = rdiv(t, a.ntn);
    tl.n0 = (t - u * (int)a.ntn.d) * 32 * NT;
    int v = rdiv(u, a.nzc);
    tl.z0 = (u - v * (int)a.nzc.d) * a.dzc;
    u = rdiv(v, a.tiles_w);
    tl.w0 = (v - u * (int)a.tiles_w.d) * TW;
    const int nb = rdiv(u, a.tiles_h);
    tl.nb = nb;
    tl.h0 = (u - nb * (int)a.tiles_h.d) * RFTH;
    tl.z1 = min(tl.z0 + a.dzc, a.y.d);
    tl.di_lo = max(0, tl.z0 - a.pd);
    tl.nsl = min(a.x.d - 1, tl.z1 + KD - 2 - a.pd) - tl.di_lo + 1;
    tl.xo = nb * a.x.sn + (tl.h0 - a.ph) * a.x.sh + (tl.w0 - a.pw) * a.x.sw;
    tl.yo = nb * a.y.sn + tl.h0 * a.y.sh + tl.w0 * a.y.sw + (SP == SP_Y ? 0 : tl.n0);
    return tl;
  };
  // spatial validity of this lane's A pieces for a tile (bit q)
  auto tile_mask = [&](const RTile& tl) __attribute__((always_inline)) {
    const int hb = tl.h0 - a.ph, wb = tl.w0 - a.pw;
    unsigned m = 0;
#pragma unroll
    for (int q = 0; q < RNQ; ++q) {
      const int hh = hwv[q] >> 8, ww = hwv[q] & 0xff;
      const bool ok = hwv[q] >= 0 && (unsigned)(hb + hh) < (unsigned)a.x.h && (unsigned)(wb + ww) < (unsigned)a.x.w;
      m |= (ok ? 1u : 0u) << q;
    }
    return m;
  };
  // kd taps with an output depth inside [z0, z1) for input slice di
  auto kd_mask = [&](int z0, int z1, int di) __attribute__((always_inline)) {
    const int P = di + a.pd;
    unsigned m = P >= z0 && P < z1 ? 1u : 0u;
    if constexpr (KD == 3) m |= (P - 1 >= z0 && P - 1 < z1 ? 2u : 0u) | (P - 2 >= z0 && P - 2 < z1 ? 4u : 0u);
    return m;
  };

  // ---- the DMA walk (two stages ahead of the compute walk) ----
  struct Walk {
    int t, sl, c;
    RTile tl;
    unsigned m;  // lane mask (VGPR)
  };
  auto advance = [&](Walk& k) __attribute__((always_inline)) -> bool {
    if (++k.c < a.nchunk) return true;
    k.c = 0;
    if (++k.sl < k.tl.nsl) return true;
    k.sl = 0;
    k.t += gx;
    if (k.t >= t_hi) return false;
    k.tl = decode(k.t);
    k.m = tile_mask(k.tl);
    return true;
  };
  const char* zp = reinterpret_cast<const char*>(g_roll_zero);
  if constexpr (ROLL_LEAN) asm volatile("" : "+v"(zp));  // keep the zero page address in VGPRs
  struct Dma {
    const H* xb;
    const H* wsrc;
    unsigned use;  // bit q: the piece reads its source (else the zero page)
  };
  // stage of walk k: A pieces of slice di, channels [c0, c0 + 16) (zero page
  // outside the image), B pieces of the weight slab (zero page for taps of a
  // kd with no output depth in the tile), and the junk pieces (zero page)
  auto prep = [&](const Walk& k) __attribute__((always_inline)) {
    Dma d;
    const int di = k.tl.di_lo + k.sl;
    const int c0 = k.c * RCH;
    d.xb = reinterpret_cast<const H*>(a.x.ptr) + (k.tl.xo + di * a.x.sd + (SP == SP_X || SP == SP_FOLD ? a.spoff[k.c] : c0));
    if constexpr (SP == SP_FOLD) {
      const int kdf = a.sptap[k.c];
      d.wsrc = reinterpret_cast<const H*>(a.w) + (k.tl.n0 * a.cin_pad + kdf * a.fold_wstride + (k.c - kdf * a.fold_nc) * RCH);
    } else {
      d.wsrc = reinterpret_cast<const H*>(a.w) + (k.tl.n0 * a.cin_pad + c0);
    }
    const unsigned km = kd_mask(k.tl.z0, k.tl.z1, di);
    d.use = (k.m & qa) | ((km & 1) ? qkd0 : 0u) | ((km & 2) ? qkd1 : 0u) | ((km & 4) ? qkd2 : 0u);
    return d;
  };
  auto dma = [&](Dma d, int q, int slot) __attribute__((always_inline)) {
    const int j = wave + RNW * q;
    const H* base = ((qa >> q) & 1) ? d.xb : d.wsrc;
    const void* src = ((d.use >> q) & 1) ? (const void*)(base + rel[q]) : (const void*)zp;
    if constexpr (!(ROLL_ABL & 2)) {
      if constexpr (ROLL_LEAN) glds16_m0(src, lds_addr(lds) + slot * RSLOT + j * 1024);
      else glds16(src, lds_addr(lds) + slot * RSLOT + j * 1024);
    }
  };

  f32x16 acc[NACC][RMS];  // KD 3: bank b holds the output depth dz with dz % 3 == b; KD 1: output block b
#pragma unroll
  for (int k = 0; k < NACC; ++k)
#pragma unroll
    for (int m = 0; m < RMS; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[k][m][i] = 0.f;

  // WR: the whole weight image of output block n0 into the resident region
  // (piece p = chunk * NB + (tap, nt); each wave issues every 8th piece)
  int wblk = -1;  // output block held by the resident region
  auto load_w = [&](int n0) __attribute__((always_inline)) {
    if constexpr (WR) {
      const int nw = a.nchunk * G::NB;
      const int co = lane >> 1;
      const int ph = (lane & 1) ^ ((co >> 3) & 1);
      for (int p = wave; p < nw; p += RNW) {
        const int c = p / G::NB, bp = p - c * G::NB;
        const int tap = bp / NT, nt = bp - tap * NT;
        const H* src = reinterpret_cast<const H*>(a.w) + ((tap * a.cout_pad + n0 + nt * 32 + co) * a.cin_pad + c * RCH + 8 * ph);
        glds16_m0(src, __builtin_amdgcn_readfirstlane(lds_addr(wres) + p * 1024));
      }
      wblk = n0;
    }
  };

  // BN-affine/ReLU prologue on this lane's own landed A piece q of slot `sl`
  // (in-image pieces; the halo stays zero as in the reference, which pads
  // relu(bn(x))): c = the stage's channel chunk, m = its lane mask.
  const bool relu_in = (a.prologue & VSRK_PRO_RELU) != 0;
  auto transform_piece = [&](char* sl, int q, int c, unsigned m) __attribute__((always_inline)) {
    const int j = wave + RNW * q;
    if (((qa & m) >> q) & 1) {
      uint4* p = reinterpret_cast<uint4*>(sl + j * 1024 + lane * 16);
      const int ww = hwv[q] & 0xff;
      *p = prologue_lds<H>(*p, c * RCH + 8 * ((lane & 1) ^ ((ww >> 3) & 1)), relu_in, lsc, lsh);
    }
  };

  // Epilogue operand prefetch (2-D: the residual or mask; 3-D: the BN input
  // of RE_BNRED), in the transposed epilogue's layout: lane l reads 8
  // channels (16 bytes) 8 (l & 3) .. +7 of the block of voxel (l >> 2) + 16 k,
  // a slice's last stages ahead of its flush.  The stage waits of the main
  // loop count them (see pf_hold) and retire them before the flush; as
  // ordinary loads the compiler also waits for them itself before their
  // first use.
  typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
  typedef u32x4_t PreT[PREF ? RMS : 1][PREF ? NT : 1][2];
  PreT pre;
  const RView& pv = (EM & RE_RES) ? a.res : a.msk;  // (RE_BNRED: msk is the BN input view)
  const int tv = lane >> 2, tc8 = lane & 3;  // transposed roles: voxel (of 16), 8-channel group
  auto load_pre = [&](PreT& dst, const RTile& tl, int dz) __attribute__((always_inline)) {
    // (ablation 2 issues no DMA, so the compile-time waits would not cover
    // these register loads: never combine them)
    if constexpr (PREF && !(ROLL_ABL & 2)) {
#pragma unroll
      for (int ms = 0; ms < RMS; ++ms) {
        const int ho = tl.h0 + wave * RMS + ms;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          // (SWAP: the lanes of epilogue_sw -- voxel (r & 15) + 16 k, chunk ecc)
          const int wo = tl.w0 + (SWAP ? (r & 15) : tv) + 16 * k;
          const bool ok = ho < a.y.h && wo < a.y.w;
          const H* pp = reinterpret_cast<const H*>(pv.ptr) +
                        (tl.nb * pv.sn + dz * pv.sd + ho * pv.sh + wo * pv.sw + tl.n0 + 8 * (SWAP ? 2 * (r >> 4) + hf : tc8));
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            const void* src = ok ? (const void*)(pp + nt * 32) : (const void*)zp;
            dst[ms][nt][k] = *reinterpret_cast<const u32x4_t*>(src);
          }
        }
      }
    }
  };
  auto prefetch = [&](const RTile& tl, int dz) __attribute__((always_inline)) { load_pre(pre, tl, dz); };
  auto settle = [&]() __attribute__((always_inline)) {
    if constexpr (PREF) {
#pragma unroll
      for (int ms = 0; ms < RMS; ++ms)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int k = 0; k < 2; ++k) asm volatile("" : "+v"(pre[ms][nt][k]));
    }
  };

  // One stage on slot SLOT.  Groups (kw, set b) in kw-major order: the 4
  // A fragments (halo rows) of a kw are read one kw ahead, the 3 B fragments
  // of a group (taps (kd_b, kh, kw) of set b: KD 3, the tap whose output
  // depth lives in bank b; KD 1, output block b) one group ahead, both
  // unconditionally (an idle kd's taps are zeros), then 3 x RMS MFMAs if set
  // b has work.  Groups 0..NQ-1 each issue one DMA piece of the stage two
  // ahead (slot SLOT+2); the remaining groups apply the BN/ReLU prologue to
  // this wave's A pieces of the NEXT stage (slot SLOT+1, landed one stage
  // ago), beside the MFMAs instead of in front of the barrier.
  auto compute = [&](auto slot_c, int P, unsigned km, Dma dn, bool don, bool tnext, int tc,
                     unsigned tm, unsigned tk0, unsigned tk1, int cchunk) __attribute__((always_inline)) {
    constexpr int SLOT = decltype(slot_c)::value;
    const char* sl = lds + SLOT * RSLOT;
    const char* bsl = WR ? wres + cchunk * G::NB * 1024 : sl;  // where this stage's B pieces are
    char* sl1 = lds + ((SLOT + 1) % 3) * RSLOT;
    const int pm = P % 3;
    uint32_t bofs[NACC];  // byte offset of set b's taps
    unsigned bm;          // sets with work
    if constexpr (KD == 3) {
#pragma unroll
      for (int b = 0; b < 3; ++b) bofs[b] = (uint32_t)(((pm + 3 - b) % 3) * 9 * 1024);
      bm = ((km & 1) ? (1u << pm) : 0u) | ((km & 2) ? (1u << ((pm + 2) % 3)) : 0u) |
           ((km & 4) ? (1u << ((pm + 1) % 3)) : 0u);
    } else {
#pragma unroll
      for (int b = 0; b < NACC; ++b) bofs[b] = (uint32_t)(b * 1024);
      bm = (km & 1) ? (1u << NACC) - 1 : 0u;
    }
    uint4 ax[2][RMS + 2];
    uint4 bw[2][3];
    if constexpr ((ROLL_ABL & 8) != 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < RMS + 2; ++j) ax[i][j] = make_uint4(lane, 1, 2, 3);
#pragma unroll
        for (int j = 0; j < 3; ++j) bw[i][j] = make_uint4(lane, 3, 2, 1);
      }
    }
    auto load_a = [&](uint4* af, int kw) __attribute__((always_inline)) {
      if constexpr (!(ROLL_ABL & 8))
#pragma unroll
        for (int hr = 0; hr < RMS + 2; ++hr) af[hr] = *reinterpret_cast<const uint4*>(sl + abase[kw] + hr * RHW * 32);
    };
    auto load_b = [&](uint4* bf, int g) __attribute__((always_inline)) {
      const int kw = g / NACC, b = g % NACC;
      const char* pb = bsl + bbase + bofs[b] + kw * NT * 1024;
      if constexpr (!(ROLL_ABL & 8))
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) bf[kh] = *reinterpret_cast<const uint4*>(pb + kh * 3 * NT * 1024);
    };
    load_a(ax[0], 0);
    load_b(bw[0], 0);
#pragma unroll
    for (int g = 0; g < G::NG; ++g) {
      const int kw = g / NACC, b = g % NACC;
      if (g + 1 < G::NG) load_b(bw[(g + 1) & 1], g + 1);
      if (b == (NACC == 3 ? 1 : 0) && kw + 1 < 3) load_a(ax[(kw + 1) & 1], kw + 1);
      if (g < G::NDG && (ROLL_LEAN || don)) {
#pragma unroll
        for (int pp = 0; pp < G::PPG; ++pp)
          if (g * G::PPG + pp < RNQ) dma(dn, g * G::PPG + pp, (SLOT + 2) % 3);
      }
      if constexpr (PRO) {
        if (g == G::NDG && tnext) {
          if (ROLL_LEAN || don) roll_wait_vmcnt<RNQ>();  // the next stage's pieces landed (the one after stays in flight)
          else roll_wait_vmcnt<0>();
        }
        if (g >= G::NDG && tnext) {
#pragma unroll
          for (int q = (g - G::NDG) * G::TPG; q < (g - G::NDG + 1) * G::TPG && q < RNA; ++q)
            transform_piece(sl1, q, tc, tm);
        }
      }
      if ((bm >> b) & 1) {
        const unsigned tkb = b == 0 ? tk0 : tk1;  // sub-pixel forms: taps of this set's phase
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          if ((SP != SP_X && SP != SP_Y) || ((tkb >> (kh * 3 + kw)) & 1)) {
#pragma unroll
            for (int ms = 0; ms < RMS; ++ms)
              if constexpr (!(ROLL_ABL & 1)) mma<H>(acc[b][ms], bw[g & 1][kh], ax[kw & 1][ms + kh]);
          }
        }
      }
    }
  };

  const float osc = a.out_scale;
  const float pslope = (EM & RE_PRELU) ? *a.act_param : 0.f;
  const float mslope = (EM & RE_PMASK) ? *a.mask_slope : 0.f;
  float sacc = 0.f;  // RE_PMASK: this lane's sum_{mask < 0} out * mask
  auto slope_out = [&](float v) __attribute__((always_inline)) {  // the wave's partial, at its end
    const double wsum = vsrk_wave_sum((double)v);
    if (lane == 0) a.slope_part[blockIdx.x * RNW + wave] = wsum;
  };
  // Transposed epilogue (output block nt of depth dz; both forms): per row ms
  // the wave parks its fp32 accumulators (32 voxels x 32 channels) in LDS and
  // reads them back as 8 consecutive channels of one voxel per lane, so every
  // global access (output, residual, mask, accumulate, the BN input of
  // RE_BNRED) is 16 contiguous bytes and a wave instruction covers 16 voxels
  // x 64 bytes -- instead of 32 voxels x 8 bytes, which doubled the cost of a
  // residual / mask operand in the 2-D form and of the BN input read in the
  // fused 3-D data gradient (2.0 vs 1.24 ms per DUF launch, round 3).
  // The scratch is the wave's own DMA pieces 0-1 of the slot the next DMA
  // fills (free after the barrier; only this wave writes them, and only after
  // its flush): a row is parked in two halves of 16 voxels, voxel v in piece
  // (v % 16) / 8, row v % 8 (128 bytes), 16-byte column c at c ^ (v & 7)
  // (conflict-free parking and read-back; 2 KB per wave fits every slot form).
  // Epilogue operand modes: EO_PRE takes the slice's prefetch; EO_LOAD loads
  // the operand synchronously -- 3-D RE_BNRED: every row's BN input at the
  // start, so a bank waits for one load latency instead of one
  // per row, each behind the stores of the rows before it (the tile-end flush
  // of the banks that were not prefetched: -6 % at DUF's F = 224 unit)
  enum { EO_LOAD = 0, EO_PRE = 1 };
  auto epilogue_tr = [&](const f32x16 (&A)[RMS], const RTile& tl, int dz, int nt, int omode, char* scr)
                         __attribute__((always_inline)) {
    const bool use_pre = omode == EO_PRE;
    char* ws = scr + wave * 1024;
    // (3-D RE_BNRED: EO_LOAD must not reuse `pre`: at the end of a tile it
    // may still hold the finishing bank's prefetched operand)
    PreT pop;
    if constexpr (PREF && KD == 3) {
      if (omode == EO_PRE) {
#pragma unroll
        for (int ms = 0; ms < RMS; ++ms)
#pragma unroll
          for (int k = 0; k < 2; ++k) pop[ms][0][k] = pre[ms][0][k];
      } else {
        load_pre(pop, tl, dz);
      }
    }
#pragma unroll
    for (int ms = 0; ms < RMS; ++ms) {
      const int ho = tl.h0 + wave * RMS + ms;
      if (ho >= a.y.h) continue;  // wave-uniform
      const int co = tl.n0 + nt * 32 + 8 * tc8;
      // (RE_BNRED: a data gradient, no bias and unit scale -- the host
      // checks -- so the bias table is not read and the scale not applied)
      constexpr bool PLAIN = (EM & RE_BNRED) != 0;
      float bsv[8];
      if constexpr (!PLAIN) {
        const float4 b0 = *reinterpret_cast<const float4*>(lbias + co);
        const float4 b1 = *reinterpret_cast<const float4*>(lbias + co + 4);
        bsv[0] = b0.x; bsv[1] = b0.y; bsv[2] = b0.z; bsv[3] = b0.w;
        bsv[4] = b1.x; bsv[5] = b1.y; bsv[6] = b1.z; bsv[7] = b1.w;
      }
      if constexpr (!PARK2) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(ws + (r >> 3) * RNW * 1024 + (r & 7) * 128 + (((2 * g + hf) ^ (r & 7)) * 16)) =
              make_float4(A[ms][4 * g], A[ms][4 * g + 1], A[ms][4 * g + 2], A[ms][4 * g + 3]);
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (PARK2 && (r >> 4) == k) {  // this half's 16 voxels park their 32 channels
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(ws + ((r >> 3) & 1) * RNW * 1024 + (r & 7) * 128 + (((2 * g + hf) ^ (r & 7)) * 16)) =
                make_float4(A[ms][4 * g], A[ms][4 * g + 1], A[ms][4 * g + 2], A[ms][4 * g + 3]);
        }
        const int v = tv + 16 * k, wo = tl.w0 + v;
        const char* rb = PARK2 ? ws + (tv >> 3) * RNW * 1024 + (tv & 7) * 128 : ws + (v >> 3) * RNW * 1024 + (v & 7) * 128;
        const float4 q0 = *reinterpret_cast<const float4*>(rb + (((2 * tc8) ^ (v & 7)) * 16));
        const float4 q1 = *reinterpret_cast<const float4*>(rb + (((2 * tc8 + 1) ^ (v & 7)) * 16));
        float t[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if constexpr (!PLAIN) t[e] = fmaf(t[e], osc, bsv[e]);
          if constexpr (EM & RE_RELU) t[e] = fmaxf(t[e], 0.f);
          if constexpr (EM & RE_PRELU) t[e] = t[e] > 0.f ? t[e] : pslope * t[e];
        }
        if (wo < a.y.w && (KD == 1 || co < a.cout)) {  // (3-D: y->c % 8 == 0, whole 8-channel groups)
          H* yp = reinterpret_cast<H*>(a.y.ptr) + (tl.yo + dz * a.y.sd + (wave * RMS + ms) * a.y.sh + v * a.y.sw +
                                                   (SP == SP_Y ? a.spoff[(tl.n0 >> 5) + nt] : nt * 32) + 8 * tc8);
          if constexpr (EM & RE_BNRED) {
            float tr[8], xb[8];
            Chunk<H>::unpack(Chunk<H>::pack(t), tr);  // the stored (rounded) dz, as the separate reduce reads it
            uint4 xv;
            if constexpr (PREF) {
              xv = __builtin_bit_cast(uint4, pop[ms][nt][k]);
            } else {
              xv = *reinterpret_cast<const uint4*>(reinterpret_cast<const H*>(a.bnx) +
                                                   (yp - reinterpret_cast<H*>(a.y.ptr)));
            }
            Chunk<H>::unpack(xv, xb);
            // scale, shift, mean of the lane's 8 channels (the sums of
            // dy' (x - mean) take invstd in the final kernel: one VALU op
            // and two LDS reads less per element chunk)
            float cst[3][8];
#pragma unroll
            for (int k4 = 0; k4 < 3; ++k4) {
              const float4 c0 = *reinterpret_cast<const float4*>(lbn + k4 * a.cout_pad + co);
              const float4 c1 = *reinterpret_cast<const float4*>(lbn + k4 * a.cout_pad + co + 4);
              cst[k4][0] = c0.x; cst[k4][1] = c0.y; cst[k4][2] = c0.z; cst[k4][3] = c0.w;
              cst[k4][4] = c1.x; cst[k4][5] = c1.y; cst[k4][6] = c1.z; cst[k4][7] = c1.w;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float dy = fmaf(xb[e], cst[0][e], cst[1][e]) > 0.f ? tr[e] : 0.f;
              rs1[e] += dy;
              rs2[e] = fmaf(dy, xb[e] - cst[2][e], rs2[e]);
            }
          }
          if constexpr (EM & RE_MASK) {
            uint4 mv;
            if constexpr (PREF) {
              if (use_pre) mv = __builtin_bit_cast(uint4, pre[ms][nt][k]);
              else
                mv = *reinterpret_cast<const uint4*>(reinterpret_cast<const H*>(a.msk.ptr) +
                                                     (tl.nb * a.msk.sn + dz * a.msk.sd + ho * a.msk.sh + wo * a.msk.sw + co));
            } else {
              mv = *reinterpret_cast<const uint4*>(reinterpret_cast<const H*>(a.msk.ptr) +
                                                   (tl.nb * a.msk.sn + dz * a.msk.sd + ho * a.msk.sh + wo * a.msk.sw + co));
            }
            float m[8];
            Chunk<H>::unpack(mv, m);
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] = m[e] > 0.f ? t[e] : 0.f;
          }
          if constexpr (EM & RE_PMASK) {
            if constexpr (EM & RE_ACC) {  // the consumer's PReLU backward sees the whole sum: after the accumulate
              float o[8];
              Chunk<H>::unpack(*reinterpret_cast<const uint4*>(yp), o);
#pragma unroll
              for (int e = 0; e < 8; ++e) t[e] += o[e];
            }
            const uint4 mv = *reinterpret_cast<const uint4*>(reinterpret_cast<const H*>(a.msk.ptr) +
                                                             (yp - reinterpret_cast<H*>(a.y.ptr)));
            float m[8];
            Chunk<H>::unpack(mv, m);
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] = m[e] > 0.f ? t[e] : mslope * t[e];
            float tr[8];
            Chunk<H>::unpack(Chunk<H>::pack(t), tr);  // the stored (rounded) values, as prelu_bwd reads them
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (m[e] < 0.f) sacc = fmaf(tr[e], m[e], sacc);
          }
          if constexpr (EM & RE_RES) {
            uint4 rv;
            if constexpr (PREF) {
              if (use_pre) rv = __builtin_bit_cast(uint4, pre[ms][nt][k]);
              else
                rv = *reinterpret_cast<const uint4*>(reinterpret_cast<const H*>(a.res.ptr) +
                                                     (tl.nb * a.res.sn + dz * a.res.sd + ho * a.res.sh + wo * a.res.sw + co));
            } else {
              rv = *reinterpret_cast<const uint4*>(reinterpret_cast<const H*>(a.res.ptr) +
                                                   (tl.nb * a.res.sn + dz * a.res.sd + ho * a.res.sh + wo * a.res.sw + co));
            }
            float rr[8];
            Chunk<H>::unpack(rv, rr);
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] += rr[e];
          }
          if constexpr ((EM & RE_ACC) && !(EM & RE_PMASK)) {
            float o[8];
            Chunk<H>::unpack(*reinterpret_cast<const uint4*>(yp), o);
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] += o[e];
          }
#if ROLL_NT
          __builtin_nontemporal_store(__builtin_bit_cast(roll_u32x4, Chunk<H>::pack(t)), reinterpret_cast<roll_u32x4*>(yp));
#else
          *reinterpret_cast<uint4*>(yp) = Chunk<H>::pack(t);
#endif
        }
      }
    }
  };
  // Register-transposed epilogue (SWAP: 2-D, no prefetched operand; output
  // block nt of depth dz).  The 32x32 accumulator of a row holds, in lane
  // (r, hf), voxel r and the channels 8 g + 4 hf + i (register 4 g + i).
  // v_permlane32_swap on the register pairs (4 g + i, 4 g + 4 + i), g = 0, 2,
  // leaves lane (r, hf) with the 8 consecutive channels 16 p + 8 hf .. +7 of
  // voxel r in registers 8 p .. +7; v_permlane16_swap on the pairs (e, 8 + e)
  // then trades the upper 16 lanes' p = 0 chunk for the lower 16 lanes' p = 1
  // chunk: lane (r, hf) ends with the 8-channel chunk ecc = 2 (r >> 4) + hf of
  // the two voxels (r & 15) + 16 q in registers 8 q .. +7.  Every global
  // access is 16 contiguous bytes (a wave instruction covers 16 whole 64-byte
  // voxel rows), as in epilogue_tr, without the LDS park and its waits; the
  // out-of-range voxels take a buffer offset past the resource (loads read
  // zero, stores are dropped).
  const int ecc = 2 * (r >> 4) + hf;
  auto epilogue_sw = [&](const f32x16 (&A)[RMS], const RTile& tl, int dz, int nt, bool use_pre) __attribute__((always_inline)) {
    const int64_t sbase = (int64_t)tl.nb * a.y.sn + (int64_t)dz * a.y.sd;
    const RRsrc ry = roll_rsrc(reinterpret_cast<const H*>(a.y.ptr) + sbase);
    // (RE_PMASK: the mask has y's geometry and strides, the host checks)
    const RRsrc rpm = roll_rsrc(reinterpret_cast<const H*>((EM & RE_PMASK) ? a.msk.ptr : a.y.ptr) + sbase);
    const RRsrc rmk = roll_rsrc(reinterpret_cast<const H*>(a.msk.ptr) + ((int64_t)tl.nb * a.msk.sn + (int64_t)dz * a.msk.sd));
    const RRsrc rrs = roll_rsrc(reinterpret_cast<const H*>(a.res.ptr) + ((int64_t)tl.nb * a.res.sn + (int64_t)dz * a.res.sd));
    const int co = tl.n0 + nt * 32 + 8 * ecc;
    const int ych = (SP == SP_Y ? a.spoff[(tl.n0 >> 5) + nt] : tl.n0 + nt * 32) + 8 * ecc;
    float bsv[8];
    {
      const float4 b0 = *reinterpret_cast<const float4*>(lbias + co);
      const float4 b1 = *reinterpret_cast<const float4*>(lbias + co + 4);
      bsv[0] = b0.x; bsv[1] = b0.y; bsv[2] = b0.z; bsv[3] = b0.w;
      bsv[4] = b1.x; bsv[5] = b1.y; bsv[6] = b1.z; bsv[7] = b1.w;
    }
#pragma unroll
    for (int ms = 0; ms < RMS; ++ms) {
      const int ho = tl.h0 + wave * RMS + ms;
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = A[ms][i];
#pragma unroll
      for (int g = 0; g < 4; g += 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, v[4 * g + i]),
                                                           __builtin_bit_cast(uint32_t, v[4 * g + 4 + i]), false, false);
          v[4 * g + i] = __builtin_bit_cast(float, (uint32_t)sw[0]);
          v[4 * g + 4 + i] = __builtin_bit_cast(float, (uint32_t)sw[1]);
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, v[e]),
                                                         __builtin_bit_cast(uint32_t, v[8 + e]), false, false);
        v[e] = __builtin_bit_cast(float, (uint32_t)sw[0]);
        v[8 + e] = __builtin_bit_cast(float, (uint32_t)sw[1]);
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {  // the voxel (r & 15) + 16 q
        const int wo = tl.w0 + (r & 15) + 16 * q;
        const bool ok = ho < a.y.h && wo < a.y.w;
        const uint32_t yoff = ok ? 2u * (uint32_t)(ho * a.y.sh + wo * a.y.sw + ych) : ROLL_OOB;
        float t[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          t[e] = fmaf(v[8 * q + e], osc, bsv[e]);
          if constexpr (EM & RE_RELU) t[e] = fmaxf(t[e], 0.f);
          if constexpr (EM & RE_PRELU) t[e] = t[e] > 0.f ? t[e] : pslope * t[e];
        }
        if constexpr (EM & RE_MASK) {
          float m[8];
          uint4 mv;
          if (PREF && use_pre) mv = __builtin_bit_cast(uint4, pre[PREF ? ms : 0][PREF ? nt : 0][q]);
          else mv = roll_bload16(rmk, ok ? 2u * (uint32_t)(ho * a.msk.sh + wo * a.msk.sw + co) : ROLL_OOB);
          Chunk<H>::unpack(mv, m);
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] = m[e] > 0.f ? t[e] : 0.f;
        }
        if constexpr (EM & RE_PMASK) {
          if constexpr (EM & RE_ACC) {  // the consumer's PReLU backward sees the whole sum: after the accumulate
            float o[8];
            Chunk<H>::unpack(roll_bload16(ry, yoff), o);
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] += o[e];
          }
          float m[8];
          Chunk<H>::unpack(roll_bload16(rpm, yoff), m);
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] = m[e] > 0.f ? t[e] : mslope * t[e];
          float tr[8];
          Chunk<H>::unpack(Chunk<H>::pack(t), tr);  // the stored (rounded) values, as prelu_bwd reads them
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (m[e] < 0.f) sacc = fmaf(tr[e], m[e], sacc);  // (m = 0 off the image)
        }
        if constexpr (EM & RE_RES) {
          float rr[8];
          uint4 rv;
          if (PREF && use_pre) rv = __builtin_bit_cast(uint4, pre[PREF ? ms : 0][PREF ? nt : 0][q]);
          else rv = roll_bload16(rrs, ok ? 2u * (uint32_t)(ho * a.res.sh + wo * a.res.sw + co) : ROLL_OOB);
          Chunk<H>::unpack(rv, rr);
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] += rr[e];
        }
        if constexpr ((EM & RE_ACC) && !(EM & RE_PMASK)) {
          float o[8];
          Chunk<H>::unpack(roll_bload16(ry, yoff), o);
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] += o[e];
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(roll_v4i, Chunk<H>::pack(t)), ry, (int)yoff, 0, 0);
      }
    }
  };
  // Flush after slice pdi of tile tl.  KD 3: the banks whose output depth
  // takes no more contributions -- dz = pdi + pd - 2 when the walk stays in
  // the tile (all = false), every bank at the end of the tile -- are stored
  // (if inside the tile's depth run) and zeroed.  KD 1: output depth pdi + pd,
  // every block.
  auto flush = [&](const RTile& tl, int pdi, bool all, bool use_pre, char* scr) __attribute__((always_inline)) {
    const int P = pdi + a.pd;
    if constexpr (KD == 3) {
      const int bdone = (P + 1) % 3;  // bank of P - 2
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        if (all || b == bdone) {
          const int dz = P - (P + 3 - b) % 3;  // the output depth in bank b
          if (!(ROLL_ABL & 4) && dz >= tl.z0 && dz < tl.z1)
            epilogue_tr(acc[b], tl, dz, 0, (use_pre && b == bdone) ? EO_PRE : EO_LOAD, scr);
#pragma unroll
          for (int m = 0; m < RMS; ++m)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[b][m][i] = 0.f;
        }
      }
      if constexpr ((EM & RE_BNRED) != 0) {
        if (all) {
          // the tile's partials: butterfly over the 16 lanes of each 8-channel
          // column (lanes with equal lane & 3; fixed order); lanes 0-3 write
          // [wave][sum: 32 channels | sum xhat: 32 channels] as 16-byte rows
#pragma unroll
          for (int i = 0; i < 8; ++i) {
#pragma unroll
            for (int off = 4; off < 64; off <<= 1) {
              rs1[i] += __shfl_xor(rs1[i], off);
              rs2[i] += __shfl_xor(rs2[i], off);
            }
          }
          if (lane < 4) {
            float4* o = reinterpret_cast<float4*>(a.red_ws + ((int64_t)tl.t * RNW + wave) * 64 + 8 * lane);
            o[0] = make_float4(rs1[0], rs1[1], rs1[2], rs1[3]);
            o[1] = make_float4(rs1[4], rs1[5], rs1[6], rs1[7]);
            o[8] = make_float4(rs2[0], rs2[1], rs2[2], rs2[3]);
            o[9] = make_float4(rs2[4], rs2[5], rs2[6], rs2[7]);
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) rs1[i] = rs2[i] = 0.f;
        }
      }
    } else {
#pragma unroll
      for (int b = 0; b < NACC; ++b) {
        if (!(ROLL_ABL & 4) && P >= tl.z0 && P < tl.z1) {
          if constexpr (SWAP) epilogue_sw(acc[b], tl, P, b, use_pre);
          else epilogue_tr(acc[b], tl, P, b, use_pre ? EO_PRE : EO_LOAD, scr);
        }
#pragma unroll
        for (int m = 0; m < RMS; ++m)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[b][m][i] = 0.f;
      }
    }
  };
  // compute walk: tile ct (decoded when the walk enters it), slice cs, chunk cc
#ifdef ROLL_STAMP
  unsigned stv0 = 0, stv1 = 0;
  int stc = -4 * ROLL_STAMP_SKIP;
  auto stamp = [&]() __attribute__((always_inline)) {
    if (stc >= 0 && stc < 128) {
      const unsigned tv = (unsigned)__builtin_amdgcn_s_memtime();
      if (stc < 64) stv0 = lane == stc ? tv : stv0;
      else stv1 = lane == stc - 64 ? tv : stv1;
    }
    ++stc;
  };
#else
  auto stamp = [&]() __attribute__((always_inline)) {};
#endif
  int t = t_lo + jb;
  if (t >= t_hi) {  // (workgroup-uniform) no tile: a zero partial, still counted
    if constexpr (EM & RE_PMASK) slope_out(0.f);
    return;
  }
  Walk nx;
  nx.t = t;
  nx.sl = 0;
  nx.c = 0;
  nx.tl = decode(t);
  nx.m = tile_mask(nx.tl);
  RTile ct = nx.tl;
  unsigned cm = nx.m;
  int cs = 0, cc = 0;
  load_w(ct.n0);  // WR: retired by the first stage's wait (it is older), visible after its barrier
  {
    const Dma d0 = prep(nx);
#pragma unroll
    for (int q = 0; q < RNQ; ++q) dma(d0, q, 0);
  }
  bool vn = advance(nx);
  if (vn) {
    const Dma d1 = prep(nx);
#pragma unroll
    for (int q = 0; q < RNQ; ++q) dma(d1, q, 1);
    vn = advance(nx);
  } else if constexpr (ROLL_LEAN) {  // zero-page pieces: the waits below count two batches
    Dma d1;
    d1.xb = nullptr;
    d1.wsrc = nullptr;
    d1.use = 0;
#pragma unroll
    for (int q = 0; q < RNQ; ++q) dma(d1, q, 1);
  }
  // the stage after the current one, for the late prologue: exists, chunk, lane mask
  bool tnext;
  int tc;
  unsigned tm;
  {
    Walk k1;
    k1.t = t; k1.sl = 0; k1.c = 0; k1.tl = ct; k1.m = cm;
    tnext = advance(k1);
    tc = k1.c;
    tm = k1.m;
  }
  __syncthreads();  // bias / prologue tables visible
  if constexpr (PRO) {  // the first stage: no earlier compute transformed it
    if (ROLL_LEAN || tnext) roll_wait_vmcnt<RNQ>();
    else roll_wait_vmcnt<0>();
#pragma unroll
    for (int q = 0; q < RNA; ++q) transform_piece(lds, q, 0, cm);
  }
  RTile ptl = ct;
  int pdi = -1;     // slice whose end is still to be flushed (-1: none)
  bool pall = false;
  bool ppre = false;  // its epilogue operand was prefetched
  // The 2-D operand prefetch of a slice is issued at the end of its third-to-
  // last stage (chunk nchunk - 3), AFTER that stage's DMA pieces, and the two
  // following steps wait with NPF more loads outstanding: the slice's last two
  // stages cover its latency, as the DMA ring's two stages of lookahead do,
  // and the step after (the flush) retires it.  Shorter slices: at chunk 0
  // (one stage of cover), or with one chunk before the last stage's pieces.
  constexpr int NPF = RMS * NT * 2;
  int pf_hold = 0;         // steps whose wait leaves the prefetch in flight
  bool pf_slice = false;   // the current slice's operand was prefetched
  // one stage; false when it was the workgroup's last
  char* fscr = lds;  // the final flush's scratch slot: the one the last stage's DMA walk left free
  auto step = [&](auto slot_c) __attribute__((always_inline)) -> bool {
    fscr = lds + ((decltype(slot_c)::value + 2) % 3) * RSLOT;
    if (PREF && pf_hold > 0) {
      --pf_hold;
      if (ROLL_LEAN || tnext) roll_wait_vmcnt<RNQ + NPF>();  // this stage landed; the next stage and the prefetch stay in flight
      else roll_wait_vmcnt<NPF>();
    } else {
      if (ROLL_LEAN || tnext) roll_wait_vmcnt<RNQ>();  // this stage landed (and any earlier prefetch); the next stays in flight
      else roll_wait_vmcnt<0>();
    }
    stamp();
    if constexpr (ROLL_ABL & 16) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // this slot ready, the previous one free
    stamp();
    // WR: the compute walk entered a tile of another output block.  Every
    // wave is past the last stage that read the old image (the barrier
    // above), so the new one is issued now, its latency covered by the flush,
    // then drained (with the next stage's pieces and any prefetch) and
    // published by a second barrier.
    bool wreload = false;
    if constexpr (WR) {
      if (ct.n0 != wblk) {
        load_w(ct.n0);
        wreload = true;
      }
    }
    if (pdi >= 0) {
      if (ppre) settle();
      flush(ptl, pdi, pall, ppre, lds + ((decltype(slot_c)::value + 2) % 3) * RSLOT);
    }
    stamp();
    if (WR && wreload) {
      roll_wait_vmcnt<0>();
      asm volatile("s_barrier" ::: "memory");
    }
    const int di = ct.di_lo + cs;
    // the output depth this slice completes: 2-D di + pd, 3-D the bank of di + pd - 2
    const int pz = KD == 3 ? di + a.pd - 2 : di + a.pd;
    const bool out_in = pz >= ct.z0 && pz < ct.z1;
    bool pf_next = false;
    if constexpr (PREF) {
      if (a.nchunk == 1) {
        if (out_in) {
          prefetch(ct, pz);
          pf_slice = true;
        }
      } else if (cc == max(a.nchunk - 3 - ROLL_PFEARLY, 0) && out_in) {
        pf_next = true;
      }
    }
    Dma dn;
    dn.xb = nullptr;
    dn.wsrc = nullptr;
    dn.use = 0;
    if (vn) dn = prep(nx);
    unsigned tk0 = 0x1ffu, tk1 = 0x1ffu;
    if constexpr (SP == SP_X) tk0 = tk1 = a.sptap[cc];
    if constexpr (SP == SP_Y) {
      tk0 = a.sptap[ct.n0 >> 5];
      tk1 = a.sptap[(ct.n0 >> 5) + 1];
    }
    compute(slot_c, di + a.pd, kd_mask(ct.z0, ct.z1, di), dn, vn, tnext, tc, tm, tk0, tk1, cc);
    stamp();
    if constexpr (PREF) {
      if (pf_next) {
        prefetch(ct, pz);
        pf_slice = true;
        pf_hold = min(2 + ROLL_PFEARLY, a.nchunk - 1);
      }
    }
    // the stage after the next one is nx's (issued just now): it becomes "next"
    tnext = vn;
    tc = nx.c;
    tm = nx.m;
    if (vn) vn = advance(nx);
    // advance the compute walk; a finished slice is flushed after the next barrier
    pdi = -1;
    if (++cc < a.nchunk) return true;
    cc = 0;
    ptl = ct;
    pdi = di;
    pall = false;
    ppre = pf_slice;
    pf_slice = false;
    if (++cs < ct.nsl) return true;
    cs = 0;
    pall = true;
    t += gx;
    if (t >= t_hi) return false;
    ct = decode(t);
    cm = tile_mask(ct);
    return true;
  };
  while (step(std::integral_constant<int, 0>{}) && step(std::integral_constant<int, 1>{}) &&
         step(std::integral_constant<int, 2>{})) {
  }
  roll_wait_vmcnt<0>();  // the last stage's prefetch
  if (ppre) settle();
  flush(ptl, pdi, true, ppre, fscr);
#ifdef ROLL_STAMP
  if (blockIdx.x < 16 && (wave == 0 || wave == 4)) {
    unsigned* o = g_roll_stamp + (blockIdx.x * 2 + (wave >> 2)) * 128;
    o[lane] = stv0;
    o[64 + lane] = stv1;
  }
#endif
  if constexpr (EM & RE_PMASK) slope_out(sacc);
}

// Channel c of the fused BN+ReLU backward reduce: the (tile, wave) partials
// of the tiles whose output block holds c (tile order: block fastest), in a
// fixed order, in double.  A (tile, wave) record is [sum: 32 | sum xhat: 32]
// over the block's channels.
__global__ __launch_bounds__(256) void roll_bnred_final_kernel(const float* __restrict__ ws, int ntiles, int ntn,
                                                               int cout, const float* __restrict__ invstd,
                                                               float* __restrict__ o1, float* __restrict__ o2) {
  const int c = blockIdx.x;
  if (c >= cout) return;
  const int blk = c >> 5, cc = c & 31;
  const int nt = (ntiles - blk + ntn - 1) / ntn;  // tiles blk, blk + ntn, ...
  double s1 = 0.0, s2 = 0.0;
  constexpr int U = 8;  // loads in flight per lane before the adds (the partials are latency-bound)
  const int n = nt * RNW;
  for (int i0 = threadIdx.x; i0 < n; i0 += 256 * U) {
    float v1[U], v2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 256 * u;
      v1[u] = v2[u] = 0.f;
      if (i < n) {
        const int t = blk + ntn * (i / RNW), w = i % RNW;
        const float* p = ws + ((int64_t)t * RNW + w) * 64;
        v1[u] = p[cc];
        v2[u] = p[32 + cc];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s1 += v1[u];
      s2 += v2[u];
    }
  }
  __shared__ double r1[256], r2[256];
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) {
      r1[threadIdx.x] += r1[threadIdx.x + k];
      r2[threadIdx.x] += r2[threadIdx.x + k];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    o1[c] = (float)r1[0];
    o2[c] = (float)(r2[0] * (double)invstd[c]);  // the partials are sums of dy' (x - mean)
  }
}


int g_roll_mode = -1;  // -1: from VSRK_CONV_ROLL (unset: 2), 0 off, 1 forced on, 2 automatic
// resident weights (WR): -1 from VSRK_ROLL_WRES (unset: 1), 0 off, 1 where
// faster, 2 also with the prefetched residual / mask epilogue (tests)
int g_roll_wr_mode = -1;

int roll_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <int KD, int NT, int PRO, int EM, int SP, typename H, int WR = 0>
int launch_roll(const RollArgs& a, size_t lds, int grid, hipStream_t s) {
  auto kern = conv_roll_kernel<KD, NT, PRO, EM, SP, H, WR>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<<<grid, RNW * 64, lds, s>>>(a);
  VSRK_LAUNCH_CHECK("conv_fwd(roll)");
  return VSRK_OK;
}


}  // namespace

#ifdef ROLL_FOLD_TU
// The depth-folded forward (this translation unit is conv_roll_fold.hip:
// ROLL_RMS 4, 32-row tiles).  DUF's last unit is Conv3d(224, 32, 3, padding
// (0, 1, 1)) over three input slices into one output depth (duf_net.py:214):
// a rolling walk finds one kd tap per staged slice, so its stage carried a
// third of the 3-D form's MFMAs beside the same 47 DMA pieces (and 27 B
// fragment reads) -- it ran on conv_fast at ~0.22 of peak.  Folded, it is a
// 3x3 conv over 3 x cin (kd, channel) chunks with one 32-channel output
// block: a stage stages 37 A pieces (34 x 34 halo voxels of 16 channels) and
// the 9 B pieces of its depth tap, and each wave runs 9 taps x 4 rows = 36
// MFMAs per stage (18 in the 3-D form's one-bank stages).
// 1 = launched, 0 = not eligible, < 0 = -(error status)
int vsrk_conv_fwd_roll_fold(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                            const float* pro_scale, const float* pro_shift, const vsrk_tensor5* y, hipStream_t s) {
  if (d->kd != 3 || d->kh != 3 || d->kw != 3 || d->pd != 0 || x->d != 3 || y->d != 1) return 0;
  if (!vsrk_is16(x->dtype) || y->dtype != x->dtype || x->shuffle > 1 || y->shuffle > 1) return 0;
  if (d->act != VSRK_ACT_NONE && d->act != VSRK_ACT_RELU) return 0;
  if (d->accumulate || d->mask_slope || d->bias_perm_r > 1) return 0;
  if (x->c % RCH != 0 || 3 * (x->c / RCH) > RMAXSUB || !chunk_ok(x, 2)) return 0;
  if (y->c % 32 != 0 || ((uintptr_t)y->ptr) % 16 != 0 || y->sn % 8 || y->sh % 8 || y->sw % 8) return 0;
  if (d->ph < 0 || d->ph > 2 || d->pw < 0 || d->pw > 2) return 0;
  if (y->h != x->h + 2 * d->ph - 2 || y->w != x->w + 2 * d->pw - 2 || y->n != x->n) return 0;
  for (const vsrk_tensor5* t : {x, y}) {  // every element offset fits in 32 bits
    const int64_t span = (int64_t)(t->n - 1) * t->sn + (int64_t)(t->d - 1) * t->sd +
                         (int64_t)(t->h + RFTH + 2) * t->sh + (int64_t)(t->w + 2 * RHW) * t->sw + t->c;
    if (span >= (1ll << 31) || t->sn < 0 || t->sd < 0 || t->sh < 0 || t->sw < 0) return 0;
  }
  RollArgs a;
  a.x.ptr = (char*)x->ptr;
  a.x.d = 1; a.x.h = x->h; a.x.w = x->w;
  a.x.sn = (int)x->sn; a.x.sd = (int)x->sd; a.x.sh = (int)x->sh; a.x.sw = (int)x->sw;
  a.y.ptr = (char*)y->ptr;
  a.y.d = 1; a.y.h = y->h; a.y.w = y->w;
  a.y.sn = (int)y->sn; a.y.sd = (int)y->sd; a.y.sh = (int)y->sh; a.y.sw = (int)y->sw;
  a.res = a.y;
  a.msk = a.y;
  a.w = w_packed;
  a.bias = bias;
  a.bias_r = 1;
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
  a.cin = 3 * x->c;
  a.cout = y->c;
  a.cin_pad = round_up(x->c, 32);  // of the packed weights
  a.cout_pad = round_up(y->c, 128);
  a.pd = 0;
  a.ph = d->ph;
  a.pw = d->pw;
  a.prologue = d->prologue;
  a.out_scale = d->out_scale;
  const int nc = x->c / RCH;
  a.nchunk = 3 * nc;
  a.fold_nc = nc;
  a.fold_wstride = 9 * a.cout_pad * a.cin_pad;
  a.fold_tab = 3 * x->c;
  a.fold_cin = x->c;
  a.act_param = nullptr;
  a.prio = 0;
  a.mask_slope = nullptr;
  a.slope_part = nullptr;
  for (int i = 0; i < a.nchunk; ++i) {
    const int kd = i / nc;
    a.spoff[i] = (int)(kd * x->sd + (i - kd * nc) * RCH);
    a.sptap[i] = (uint16_t)kd;
  }
  const int tiles_h = ceil_div(y->h, RFTH), tiles_w = ceil_div(y->w, TW), ntn = ceil_div(y->c, 32);
  const int64_t ntiles = (int64_t)y->n * tiles_h * tiles_w * ntn;
  if (ntiles == 0) return 1;
  VSRK_CHECK(ntiles < (1ll << 31), "conv_fwd(roll fold): too many tiles");
  a.dzc = 1;
  a.ntn = make_rdiv(ntn);
  a.nzc = make_rdiv(1);
  a.tiles_w = make_rdiv(tiles_w);
  a.tiles_h = make_rdiv(tiles_h);
  a.ntiles = (int)ntiles;
  using G = RollGeo<1, 1>;
  const size_t tables = (size_t)a.cout_pad * 4 + (d->prologue ? 2 * (size_t)a.fold_tab * 4 : 0);
  const size_t lds = (size_t)RNSLOT * G::SLOT + tables;
  if (lds > 160 * 1024) return 0;
  const int grid = (int)vsrk_capped_grid(std::min<int64_t>(ntiles, roll_num_cus()));
  const bool relu = d->act == VSRK_ACT_RELU;
  int rc = vsrk_dispatch16(x->dtype, [&](auto tag) {
    using H = decltype(tag);
    if (d->prologue)
      return relu ? launch_roll<1, 1, 1, RE_RELU, SP_FOLD, H>(a, lds, grid, s) : launch_roll<1, 1, 1, 0, SP_FOLD, H>(a, lds, grid, s);
    return relu ? launch_roll<1, 1, 0, RE_RELU, SP_FOLD, H>(a, lds, grid, s) : launch_roll<1, 1, 0, 0, SP_FOLD, H>(a, lds, grid, s);
  });
  if (rc == VSRK_ERR_UNSUPPORTED) return 0;
  return rc == VSRK_OK ? 1 : -rc;
}
#else  // ROLL_FOLD_TU

// > 0: output depths per tile of both rolling kernels (test knob), 0: automatic
int vsrk_g_roll_dz = 0;

extern "C" int vsrk_conv_set_roll_depth(int32_t depths) {
  VSRK_CHECK(depths >= 0, "conv_set_roll_depth: depths must be >= 0");
  vsrk_g_roll_dz = depths;
  return VSRK_OK;
}

void vsrk_conv_set_roll_wr_mode(int mode) { g_roll_wr_mode = mode; }

void vsrk_conv_set_roll_mode(int mode) { g_roll_mode = mode; }

// the depth-folded form for one output depth from three slices: -1 from
// VSRK_ROLL_FOLD (unset: on), 0 off, 1 on
int g_roll_fold_mode = -1;
void vsrk_conv_set_roll_fold_mode(int mode) { g_roll_fold_mode = mode; }

// 1 = launched, 0 = not eligible, < 0 = -(error status)
size_t vsrk_roll_slope_ws_bytes() { return (size_t)roll_num_cus() * RNW * sizeof(double); }

static int roll_fwd_one(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                        const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                        const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s, const vsrk_slope_out* slope,
                        vsrk_roll_bnred* bnred);

// The rolling kernels address their views with 32-bit element offsets.  A
// batch whose views span more (DUF's 256-channel concat buffer at cfg 5:
// 128 windows x 7 x 128 x 128 x 256 = 3.8e9 elements) is launched in sample
// chunks that fit, for the forms without a cross-sample reduction (the BN
// reduce and the PReLU slope partials are per launch); before, such a
// batch fell back to conv_fast.
int vsrk_conv_fwd_roll(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                       const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                       const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s, const vsrk_slope_out* slope,
                       vsrk_roll_bnred* bnred) {
  auto span = [](const vsrk_tensor5* t, int64_t n) -> int64_t {  // as roll_fwd_one's check, for n samples
    const int64_t r = t->shuffle > 1 ? t->shuffle : 1;
    return (n - 1) * t->sn + (int64_t)(t->d - 1) * t->sd + (int64_t)(r * (t->h + RFTH + 2) - 1) * t->sh +
           (int64_t)(r * (t->w + 2 * RHW) - 1) * t->sw + t->c;
  };
  const vsrk_tensor5* ts[4] = {x, y, residual, mask};
  auto fits = [&](int64_t n) {
    for (const vsrk_tensor5* t : ts)
      if (t && span(t, n) >= (1ll << 31)) return false;
    return true;
  };
  if (slope || bnred || x->n <= 1 || y->n != x->n || fits(x->n))
    return roll_fwd_one(d, x, w_packed, bias, pro_scale, pro_shift, residual, mask, y, s, slope, bnred);
  for (const vsrk_tensor5* t : ts)
    if (t && (t->n != x->n || t->sn < 0)) return 0;
  int nc = x->n;
  while (nc > 1 && !fits(nc)) nc = (nc + 1) / 2;
  if (!fits(nc)) return 0;
  for (int n0 = 0; n0 < x->n; n0 += nc) {
    vsrk_tensor5 c[4];
    for (int i = 0; i < 4; ++i) {
      if (!ts[i]) continue;
      c[i] = *ts[i];
      c[i].n = std::min(nc, x->n - n0);
      c[i].ptr = (char*)ts[i]->ptr + (int64_t)n0 * ts[i]->sn * vsrk_esize(ts[i]->dtype);
    }
    const int rc = roll_fwd_one(d, &c[0], w_packed, bias, pro_scale, pro_shift, residual ? &c[2] : nullptr,
                                mask ? &c[3] : nullptr, &c[1], s, nullptr, nullptr);
    if (rc == 0 && n0 == 0) return 0;  // not eligible: nothing launched
    if (rc == 0) return -VSRK_ERR_INVALID;  // (same shapes, fewer samples: cannot happen)
    if (rc < 0) return rc;
  }
  return 1;
}

static int roll_fwd_one(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed, const float* bias,
                        const float* pro_scale, const float* pro_shift, const vsrk_tensor5* residual,
                        const vsrk_tensor5* mask, const vsrk_tensor5* y, hipStream_t s, const vsrk_slope_out* slope,
                        vsrk_roll_bnred* bnred) {
  if (g_roll_mode < 0) {
    const char* e = getenv("VSRK_CONV_ROLL");
    g_roll_mode = !e ? 2 : (e[0] == '0' ? 0 : 1);
  }
  if (g_roll_fold_mode < 0) {
    const char* e = getenv("VSRK_ROLL_FOLD");
    g_roll_fold_mode = (e && e[0] == '0') ? 0 : 1;
  }
  if (g_roll_mode == 0) return 0;
  if (!vsrk_is16(x->dtype) || y->dtype != x->dtype) return 0;
  if (d->kh != 3 || d->kw != 3) return 0;
  // the two forms: Conv3d 3x3x3 (32-channel output blocks) and 3x3 over
  // depth-1 slices with 64-channel output blocks (cout a multiple of 64)
  const bool k3 = d->kd == 3;
  if (!k3 && !(d->kd == 1 && d->pd == 0 && y->c % 64 == 0)) return 0;
  // PReLU-backward mask (slope): the mask has y's geometry and strides
  const bool pmask = slope != nullptr;
  if ((d->bias_perm_r > 1 && (y->shuffle != d->bias_perm_r || y->c % (d->bias_perm_r * d->bias_perm_r))) ||
      (d->mask_slope && !pmask))
    return 0;
  if (pmask) {
    if (!mask || !d->mask_slope || residual || d->kd != 1 || d->prologue) return 0;
    if (mask->dtype != y->dtype || mask->shuffle != y->shuffle || mask->n != y->n || mask->d != y->d ||
        mask->h != y->h || mask->w != y->w || mask->c != y->c || mask->sn != y->sn ||
        (y->d > 1 && mask->sd != y->sd) ||
        mask->sh != y->sh || mask->sw != y->sw)
      return 0;
  }
  if (d->act == VSRK_ACT_PRELU && (k3 || !d->act_param)) return 0;
  if (k3 && (residual || mask || d->accumulate)) return 0;
  // a single output depth from three slices (DUF's last unit): the depth-
  // folded 2-D form (conv_roll_fold.hip)
  if (k3 && y->d == 1 && x->d == 3 && d->pd == 0 && !bnred && !residual && !mask && !pmask && g_roll_fold_mode != 0) {
    if (const int rf = vsrk_conv_fwd_roll_fold(d, x, w_packed, bias, pro_scale, pro_shift, y, s)) return rf;
  }
  // automatic mode: a single output depth has no slice reuse to roll over;
  // the per-kd-stage kernel is faster there (DUF's last unit, 3 -> 1 slices
  // at F = 224: 817 vs 943 us, r3p microbench)
  if (g_roll_mode == 2 && k3 && y->d == 1 && !bnred && vsrk_g_roll_dz == 0) return 0;
  if (bnred) {
    const vsrk_tensor5* b = bnred->bnx;
    if (!k3 || d->prologue || d->act != VSRK_ACT_NONE || bias || d->out_scale != 1.f || !b || b->dtype != y->dtype ||
        b->shuffle > 1 ||
        b->n != y->n || b->d != y->d || b->h != y->h || b->w != y->w || b->c != y->c || b->sn != y->sn ||
        b->sd != y->sd || b->sh != y->sh || b->sw != y->sw)
      return 0;
  }
  // sub-pixel operands (2-D only, one of x / y): each 16-channel input chunk
  // (x) or 32-channel output block (y) must lie inside one phase
  const int sp = x->shuffle > 1 ? SP_X : (y->shuffle > 1 ? SP_Y : SP_NONE);
  if (x->shuffle > 1 && y->shuffle > 1) return 0;
  if (sp != SP_NONE) {
    if (k3 || d->prologue || residual || (mask && !pmask)) return 0;
    const vsrk_tensor5* t = sp == SP_X ? x : y;
    const int r = t->shuffle, cph = t->c / (r * r);
    if (cph * r * r != t->c || cph % (sp == SP_X ? RCH : 32) != 0) return 0;
    if (t->c / (sp == SP_X ? RCH : 32) > RMAXSUB) return 0;
  }
  if (x->c % RCH != 0 || !chunk_ok(x, 2)) return 0;
  if (d->pd < 0 || d->pd > 2 || d->ph < 0 || d->ph > 2 || d->pw < 0 || d->pw > 2) return 0;
  if (y->d != x->d + 2 * d->pd - (d->kd - 1) || y->h != x->h + 2 * d->ph - 2 || y->w != x->w + 2 * d->pw - 2) return 0;
  auto out_ok = [&](const vsrk_tensor5* t) {  // 8-byte epilogue accesses, the output's geometry
    return t->dtype == y->dtype && (t->shuffle <= 1 || (t == y && sp == SP_Y)) && t->n == y->n && t->d == y->d &&
           t->h == y->h && t->w == y->w &&
           t->c == y->c && ((uintptr_t)t->ptr) % 8 == 0 && t->sn % 4 == 0 && t->sd % 4 == 0 && t->sh % 4 == 0 &&
           t->sw % 4 == 0;
  };
  if (y->c % (k3 ? 8 : 4) != 0 || !out_ok(y)) return 0;
  if ((residual && !out_ok(residual)) || (mask && !pmask && !out_ok(mask))) return 0;
  for (const vsrk_tensor5* t : {x, y, residual, mask}) {  // every element offset fits in 32 bits
    if (!t) continue;
    const int64_t r = t->shuffle > 1 ? t->shuffle : 1;
    const int64_t span = (int64_t)(t->n - 1) * t->sn + (int64_t)(t->d - 1) * t->sd +
                         (int64_t)(r * (t->h + RFTH + 2) - 1) * t->sh + (int64_t)(r * (t->w + 2 * RHW) - 1) * t->sw +
                         t->c;
    if (span >= (1ll << 31) || t->sn < 0 || t->sd < 0 || t->sh < 0 || t->sw < 0) return 0;
  }
  // a shuffled view walks the low-res grid: its row / column strides are r
  // physical rows / columns (the phase lives in the channel offset table)
  auto rview = [](const vsrk_tensor5* t) {
    RView v;
    const int r = t->shuffle > 1 ? t->shuffle : 1;
    v.ptr = (char*)t->ptr;
    v.d = t->d; v.h = t->h; v.w = t->w;
    v.sn = (int)t->sn; v.sd = (int)t->sd; v.sh = (int)(r * t->sh); v.sw = (int)(r * t->sw);
    return v;
  };
  RollArgs a;
  a.x = rview(x);
  a.y = rview(y);
  a.res = rview(residual ? residual : y);
  a.msk = rview(mask ? mask : y);
  a.w = w_packed;
  a.bias = bias;
  a.bias_r = d->bias_perm_r > 1 ? d->bias_perm_r : 1;
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
  a.cin = x->c;
  a.cout = y->c;
  a.cin_pad = round_up(x->c, 32);
  a.cout_pad = round_up(y->c, 128);
  a.pd = d->pd;
  a.ph = d->ph;
  a.pw = d->pw;
  a.prologue = d->prologue;
  a.out_scale = d->out_scale;
  a.nchunk = x->c / RCH;
  a.act_param = d->act_param;
  {
    static int prio = -1;
    if (prio < 0) {
      const char* e = getenv("VSRK_ROLL_PRIO");
      prio = (e && e[0] == '1') ? 1 : 0;
    }
    a.prio = prio;
  }
  if (sp != SP_NONE) {
    const vsrk_tensor5* t = sp == SP_X ? x : y;
    const int r = t->shuffle, cph = t->c / (r * r), step = sp == SP_X ? RCH : 32;
    for (int i = 0; i < t->c / step; ++i) {
      const int c = i * step, sub = c / cph, cc = c - sub * cph;
      a.spoff[i] = (int)((sub / r) * t->sh + (sub % r) * t->sw + cc);
      a.sptap[i] = subpixel_tapmask(d->subpixel, r, sub);
    }
  }
  const int nt = k3 ? 1 : 2;
  const int tiles_h = ceil_div(y->h, RFTH), tiles_w = ceil_div(y->w, TW), ntn = ceil_div(y->c, 32 * nt);
  const int64_t spatial = (int64_t)y->n * tiles_h * tiles_w * ntn;
  if (spatial == 0 || y->d == 0) return 1;
  // Depth run per tile: as long as possible (each input slice then serves
  // three output depths) while the grid still gets >= 2 tiles per CU.
  int dzc = y->d;
  if (vsrk_g_roll_dz > 0) {
    dzc = std::min(vsrk_g_roll_dz, y->d);
  } else if (k3) {
    const int64_t want = 2 * (int64_t)roll_num_cus();
    if (spatial < want) {
      const int64_t runs = std::min<int64_t>(ceil_div64(want, spatial), y->d);
      dzc = (int)ceil_div64(y->d, runs);
    }
  } else {
    dzc = 1;  // 2-D: a tile is one slice
  }
  a.dzc = dzc;
  const int nzc = ceil_div(y->d, dzc);
  a.ntn = make_rdiv(ntn);
  a.nzc = make_rdiv(nzc);
  a.tiles_w = make_rdiv(tiles_w);
  a.tiles_h = make_rdiv(tiles_h);
  const int64_t ntiles = spatial * nzc;
  VSRK_CHECK(ntiles < (1ll << 31), "conv_fwd(roll): too many tiles");
  a.ntiles = (int)ntiles;
  // resident weights (WR): plain views, no prologue, the weight image of an
  // output block <= 80 KB, and (2-D) one output block for the whole launch
  // -- EDSR's 64 -> 64 body convs -- or (3-D) whole-depth tiles, where a
  // reload per tile is amortised over nsl x nchunk stages (DUF's data
  // gradients 32 -> F).  VSRK_ROLL_WRES=0 turns it off (A/B).
  if (g_roll_wr_mode < 0) {
    const char* e = getenv("VSRK_ROLL_WRES");
    g_roll_wr_mode = (e && e[0] == '0') ? 0 : 1;
  }
  const int wres_mode = g_roll_wr_mode;
  const size_t nb = k3 ? RollGeo<3, 1>::NB : RollGeo<1, 2>::NB;
  const size_t wbytes = (size_t)a.nchunk * nb * 1024;
  const size_t tables = (size_t)a.cout_pad * 4 + (d->prologue || bnred ? 2 * (size_t)a.cin_pad * 4 : 0) +
                        (bnred ? 4 * (size_t)a.cout_pad * 4 : 0);
  const size_t wslot = k3 ? RollGeo<3, 1, 1>::SLOT : RollGeo<1, 2, 1>::SLOT;
  // (2-D: not with a prefetched residual / mask operand unless forced (mode
  // 2): correct -- tests/test_roll_gpu.py compares the forced form bitwise
  // with the streamed one; round 4's wrong results came with the inline-asm
  // prefetch, whose registers the compiler could re-use before the data
  // landed, since removed -- but slower: EDSR res 129 -> 146 us, mask
  // 147 -> 163 us per launch (profiles/r5_roll_wr_prefetch_ab.txt))
  const bool pref2d =
      wres_mode != 2 && !k3 && ((residual != nullptr) != (mask != nullptr && !pmask)) && !d->accumulate;
  const bool wr = wres_mode && sp == SP_NONE && !d->prologue && wbytes <= 80 * 1024 && !pref2d &&
                  (k3 ? dzc == y->d : ntn == 1) && (size_t)RNSLOT * wslot + wbytes + tables <= 160 * 1024;
  const size_t slot = wr ? wslot : (k3 ? RollGeo<3, 1>::SLOT : RollGeo<1, 2>::SLOT);
  const size_t lds = (size_t)RNSLOT * slot + (wr ? wbytes : 0) + tables;
  if (bnred) {
    if (bnred->ws_floats < (size_t)ntiles * RNW * 64) return 0;
    a.bnx = (const char*)bnred->bnx->ptr;
    a.msk = rview(bnred->bnx);  // the epilogue operand prefetch reads the BN input through msk
    a.bn_sc = bnred->scale;
    a.bn_sh = bnred->shift;
    a.bn_mu = bnred->mean;
    a.bn_is = bnred->invstd;
    a.red_ws = bnred->ws;
    bnred->ntiles = (int)ntiles;
    bnred->ntn = ntn;
  }
  if (lds > 160 * 1024) return 0;
  const int grid = (int)vsrk_capped_grid(std::min<int64_t>(ntiles, roll_num_cus()));
  const bool relu = d->act == VSRK_ACT_RELU;
  const int em = (residual ? RE_RES : 0) | (mask ? (pmask ? RE_PMASK : RE_MASK) : 0) | (d->accumulate ? RE_ACC : 0) |
                 (relu ? RE_RELU : 0) | (d->act == VSRK_ACT_PRELU ? RE_PRELU : 0);
  a.mask_slope = d->mask_slope;
  if (pmask) {
    if ((size_t)grid * RNW > slope->cap) return 0;
    a.slope_part = slope->part;
    *slope->nparts = grid * RNW;
  }
  int rc = vsrk_dispatch16(x->dtype, [&](auto tag) {
    using H = decltype(tag);
    if (k3) {
      if (bnred)
        return wr ? launch_roll<3, 1, 0, RE_BNRED, SP_NONE, H, 1>(a, lds, grid, s)
                  : launch_roll<3, 1, 0, RE_BNRED, SP_NONE, H>(a, lds, grid, s);
      if (d->prologue) return relu ? launch_roll<3, 1, 1, RE_RELU, SP_NONE, H>(a, lds, grid, s) : launch_roll<3, 1, 1, 0, SP_NONE, H>(a, lds, grid, s);
      if (wr)
        return relu ? launch_roll<3, 1, 0, RE_RELU, SP_NONE, H, 1>(a, lds, grid, s)
                    : launch_roll<3, 1, 0, 0, SP_NONE, H, 1>(a, lds, grid, s);
      return relu ? launch_roll<3, 1, 0, RE_RELU, SP_NONE, H>(a, lds, grid, s) : launch_roll<3, 1, 0, 0, SP_NONE, H>(a, lds, grid, s);
    }
    // 2-D forms of the EDSR body and its backward: plain, ReLU, residual,
    // ReLU mask, residual + accumulate; DUF's tail conv (1,3,3) 256 -> 256
    // with the BN+ReLU prologue (duf_net.py:116-118); DRF's sub-pixel
    // projections: plain, PReLU, accumulate over a shuffled input or output
    if (d->prologue) {
      if (sp != SP_NONE || em != 0) return (int)VSRK_ERR_UNSUPPORTED;
      return launch_roll<1, 2, 1, 0, SP_NONE, H>(a, lds, grid, s);
    }
    if (sp == SP_X) {
      switch (em) {
        case 0: return launch_roll<1, 2, 0, 0, SP_X, H>(a, lds, grid, s);
        case RE_PRELU: return launch_roll<1, 2, 0, RE_PRELU, SP_X, H>(a, lds, grid, s);
        case RE_ACC: return launch_roll<1, 2, 0, RE_ACC, SP_X, H>(a, lds, grid, s);
        case RE_PMASK: return launch_roll<1, 2, 0, RE_PMASK, SP_X, H>(a, lds, grid, s);
        case RE_PMASK | RE_ACC: return launch_roll<1, 2, 0, RE_PMASK | RE_ACC, SP_X, H>(a, lds, grid, s);
        default: return (int)VSRK_ERR_UNSUPPORTED;
      }
    }
    if (sp == SP_Y) {
      switch (em) {
        case 0: return launch_roll<1, 2, 0, 0, SP_Y, H>(a, lds, grid, s);
        case RE_PRELU: return launch_roll<1, 2, 0, RE_PRELU, SP_Y, H>(a, lds, grid, s);
        case RE_ACC: return launch_roll<1, 2, 0, RE_ACC, SP_Y, H>(a, lds, grid, s);
        case RE_PMASK: return launch_roll<1, 2, 0, RE_PMASK, SP_Y, H>(a, lds, grid, s);
        case RE_PMASK | RE_ACC: return launch_roll<1, 2, 0, RE_PMASK | RE_ACC, SP_Y, H>(a, lds, grid, s);
        default: return (int)VSRK_ERR_UNSUPPORTED;
      }
    }
    if (wr) {
      switch (em) {
        case 0: return launch_roll<1, 2, 0, 0, SP_NONE, H, 1>(a, lds, grid, s);
        case RE_RELU: return launch_roll<1, 2, 0, RE_RELU, SP_NONE, H, 1>(a, lds, grid, s);
        case RE_RES | RE_ACC: return launch_roll<1, 2, 0, RE_RES | RE_ACC, SP_NONE, H, 1>(a, lds, grid, s);
        case RE_PMASK: return launch_roll<1, 2, 0, RE_PMASK, SP_NONE, H, 1>(a, lds, grid, s);
        default: return (int)VSRK_ERR_UNSUPPORTED;
      }
    }
    switch (em) {
      case 0: return launch_roll<1, 2, 0, 0, SP_NONE, H>(a, lds, grid, s);
      case RE_RELU: return launch_roll<1, 2, 0, RE_RELU, SP_NONE, H>(a, lds, grid, s);
      case RE_RES: return launch_roll<1, 2, 0, RE_RES, SP_NONE, H>(a, lds, grid, s);
      case RE_MASK: return launch_roll<1, 2, 0, RE_MASK, SP_NONE, H>(a, lds, grid, s);
      case RE_RES | RE_ACC: return launch_roll<1, 2, 0, RE_RES | RE_ACC, SP_NONE, H>(a, lds, grid, s);
      case RE_PMASK: return launch_roll<1, 2, 0, RE_PMASK, SP_NONE, H>(a, lds, grid, s);
      default: return (int)VSRK_ERR_UNSUPPORTED;
    }
  });
  if (rc == VSRK_ERR_UNSUPPORTED) return 0;
  return rc == VSRK_OK ? 1 : -rc;
}

#ifdef ROLL_STAMP
extern "C" int vsrk_roll_stamps(unsigned* dst) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_roll_stamp), sizeof(g_roll_stamp)) == hipSuccess ? 0 : 1;
}
#endif

extern "C" size_t vsrk_conv_prelu_bwd_workspace(void) {
  return std::max(vsrk_roll_slope_ws_bytes(), vsrk_pw_pbwd_ws_bytes());
}

extern "C" int vsrk_conv_fwd_prelu_bwd(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed,
                                       const float* bias, const vsrk_tensor5* y_fwd, const vsrk_tensor5* y,
                                       int32_t c_lo, float* da, int32_t accumulate_da, void* workspace,
                                       size_t workspace_bytes, void* stream) {
  VSRK_CHECK(d && x && y && y_fwd && w_packed && d->mask_slope, "conv_fwd_prelu_bwd: null argument");
  VSRK_CHECK(workspace && workspace_bytes >= vsrk_conv_prelu_bwd_workspace(),
             "conv_fwd_prelu_bwd: workspace %zu < %zu bytes", workspace_bytes, vsrk_conv_prelu_bwd_workspace());
  VSRK_CHECK(((uintptr_t)workspace & 15) == 0, "conv_fwd_prelu_bwd: workspace must be 16-byte aligned");
  VSRK_CHECK(c_lo >= 0 && c_lo < y->c, "conv_fwd_prelu_bwd: c_lo %d outside [0, %d)", c_lo, y->c);
  hipStream_t s = (hipStream_t)stream;
  if ((int64_t)y->n * y->d * y->h * y->w == 0) {  // nothing to launch: no slope gradient
    if (da && !accumulate_da) (void)hipMemsetAsync(da, 0, sizeof(float), s);
    return VSRK_OK;
  }
  int nparts = 0;
  const vsrk_slope_out so{(double*)workspace, workspace_bytes / sizeof(double), &nparts};
  int rc;
  if (d->kd == 1 && d->kh == 1 && d->kw == 1) {
    // pointwise: the staged kernel's post-accumulate form, any channel tail
    if (bias) return VSRK_ERR_UNSUPPORTED;
    rc = vsrk_conv_fwd_pw_pbwd(d, x, w_packed, y_fwd, y, c_lo, &so, s);
  } else {
    if (c_lo != 0) return VSRK_ERR_UNSUPPORTED;  // the rolling kernel masks every output channel
    rc = vsrk_conv_fwd_roll(d, x, w_packed, bias, nullptr, nullptr, nullptr, y_fwd, y, s, &so);
  }
  if (rc == 0) return VSRK_ERR_UNSUPPORTED;
  if (rc < 0) return -rc;
  if (da) {  // (da == NULL: the partials stay in the workspace slot, vsrk_slope_final_sum later)
    vsrk_slope_final((const double*)workspace, nparts, d->mask_slope, da, accumulate_da, 0, s);
    VSRK_LAUNCH_CHECK("conv_fwd_prelu_bwd_final");
  }
  return VSRK_OK;
}

int vsrk_roll_bnred_final(const vsrk_roll_bnred& r, int cout, float* sum_dy, float* sum_dy_xhat, hipStream_t s) {
  roll_bnred_final_kernel<<<cout, 256, 0, s>>>(r.ws, r.ntiles, r.ntn, cout, r.invstd, sum_dy, sum_dy_xhat);
  VSRK_LAUNCH_CHECK("conv_fwd_reduce(roll) final");
  return VSRK_OK;
}

size_t vsrk_roll_bnred_ws_floats(const vsrk_tensor5* y) {  // every depth its own tile run (an upper bound)
  return (size_t)y->n * ceil_div(y->h, RFTH) * ceil_div(y->w, TW) * ceil_div(y->c, 32) * std::max(y->d, 1) * RNW * 64;
}
#endif  // ROLL_FOLD_TU

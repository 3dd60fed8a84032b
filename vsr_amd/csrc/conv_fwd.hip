// Implicit-GEMM convolution forward / data-gradient on CDNA4 MFMA (gfx950).
//
// Replaces the nn.Conv2d / nn.Conv3d forward and backward the reference runs on
// every train step (edsr_net.py:28-64, duf_net.py:35-49,116-214,
// drf_net.py:55-147; backward via loss.backward(), base_trainer.py:128).
//
// Layout: activations channels-last (N,D,H,W,C) in bf16 or fp32; weights
// pre-packed [kd][kh][kw][cout_pad][cin_pad].  One workgroup (8 waves) owns an
// output tile of (8*MS) rows x 32 columns of one (n, d) slice and NT output
// channels.  Per (kd, 32-channel chunk) stage the input tile plus its halo is
// staged into LDS (80-byte rows: 64 data + 16 pad, conflict-free for
// ds_read_b128 column slices) and the stage's weights by LDS-DMA (64-byte
// rows, XOR-swizzled), then all KK*KK taps run out of LDS.  MFMA orientation
// is "weights x voxels" so that each lane's accumulator column is one voxel
// and its registers hold 4 consecutive output channels -> 8/16-byte
// channels-last stores.
//   bf16: v_mfma_f32_32x32x16_bf16, one per 16 channels.
//   fp32: v_mfma_f32_32x32x2_f32, four per 8 channels (exact fp32, parity path).
#include "conv_common.h"

namespace {
using namespace vsrk_conv;

// ---------------------------------------------------------------------------
// forward / data-gradient
// ---------------------------------------------------------------------------
// Persistent: a workgroup walks a run of output tiles (runs are grouped per
// XCD so concurrently processed tiles are neighbours sharing halo rows and
// weight slices in one L2).  Its work is a flat sequence of stages
// (tile, kd tap, 32-channel chunk).  While the MFMAs of stage g run, the input
// chunks of stage g+1 are loading into registers (unconditional loads from
// clamped addresses, validity applied on commit) and its weights are landing
// in the other half of a double-buffered LDS weight area by LDS-DMA — across
// tile boundaries too, so only the very first stage of a workgroup is
// exposed.  A tile's epilogue runs right after its last stage's MFMAs (no LDS
// use) and overlaps other waves' compute.  KK is a template parameter so the
// tap loop is straight-line code (LDS reads pipelined, rows shared by
// neighbouring taps read once).
template <typename T, int NT, int MS, int KK, bool VEC, typename YT>
__global__ __launch_bounds__(NTHR) void conv_fwd_kernel(ConvArgs a) {
  constexpr int NS = NT / 32;
  constexpr int FTH = 8 * MS;  // tile rows: MS rows (of 32 voxels) per wave
  constexpr int E = Chunk<T>::E;
  constexpr int CK = 4 * E;  // channels per stage: 64 bytes
  constexpr int HWd = TW + KK - 1;
  constexpr int SLOTS = (FTH + KK - 1) * HWd;
  constexpr int MAXA = (SLOTS * 4 + NTHR - 1) / NTHR;
  constexpr int TAPS = KK * KK;
  constexpr int NBI = TAPS * NT / 16;  // 1 KiB LDS-DMA wave-instructions per stage
  constexpr int BBYTES = TAPS * NT * 64;
  static_assert(MS == 1 || MS == 2, "rows per wave");
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hf = lane >> 5;
  char* ldsA = lds;
  char* ldsB = lds + SLOTS * ROWB;  // two buffers of BBYTES
  float* lsc = reinterpret_cast<float*>(ldsB + 2 * BBYTES);
  float* lsh = lsc + a.cin_pad;
  const bool relu_in = (a.prologue & VSRK_PRO_RELU) != 0;
  if (a.prologue) stage_prologue(lsc, lsh, a.prologue, a.pro_scale, a.pro_shift, a.cin, a.cin_pad, tid, NTHR);

  // this workgroup's tiles: XCD group x = blockIdx % 8 owns a contiguous
  // range of tiles; its workgroups take them round-robin.
  const int G = gridDim.x;
  const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int gx = (G >> 3) + (x < (G & 7) ? 1 : 0);  // workgroups in this XCD group
  const int t_lo = (int)((int64_t)a.ntiles * x / 8), t_hi = (int)((int64_t)a.ntiles * (x + 1) / 8);
  const int nchunk = (a.cin + CK - 1) / CK;

  struct Tile {
    int nb, dz, h0, w0, n0, kd_lo, nst;
  };
  auto decode = [&](int t) __attribute__((always_inline)) {
    Tile tl;
    const int tn = t % a.ntn;
    int tm = t / a.ntn;
    const int tw_i = tm % a.tiles_w;
    tm /= a.tiles_w;
    const int th_i = tm % a.tiles_h;
    tm /= a.tiles_h;
    tl.dz = tm % a.y.d;
    tl.nb = tm / a.y.d;
    tl.h0 = th_i * FTH;
    tl.w0 = tw_i * TW;
    tl.n0 = tn * NT;
    tl.kd_lo = max(0, a.pd - tl.dz);
    const int kd_hi = min(a.kd, a.x.d + a.pd - tl.dz);
    tl.nst = max(1, kd_hi - tl.kd_lo) * nchunk;
    return tl;
  };

  uint4 ra[MAXA];
  unsigned okmask = 0;
  auto issue = [&](const Tile& tl, int s, int buf) __attribute__((always_inline)) {
    const int kdi = tl.kd_lo + s / nchunk;
    const int c0 = (s % nchunk) * CK;
    const int di = tl.dz + kdi - a.pd;
    const bool dvalid = di >= 0 && di < a.x.d;
    okmask = 0;
#pragma unroll
    for (int i = 0; i < MAXA; ++i) {
      const int q = tid + i * NTHR;
      const int slot = q >> 2;
      const int hh = slot / HWd, ww = slot - hh * HWd;
      const int hi = tl.h0 + hh - a.ph, wi = tl.w0 + ww - a.pw;
      const int c = c0 + (q & 3) * E;
      const bool ok = q < SLOTS * 4 && dvalid && hi >= 0 && hi < a.x.h && wi >= 0 && wi < a.x.w && c < a.cin;
      okmask |= (ok ? 1u : 0u) << i;
      if constexpr (VEC) {
        ra[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.x.ptr) +
                                                view_off(a.x, tl.nb, ok ? di : 0, ok ? hi : 0, ok ? wi : 0,
                                                         ok ? c : 0));
      } else {
        ra[i] = ok ? load_raw<T>(a.x, tl.nb, di, hi, wi, c, a.cin, false) : make_uint4(0, 0, 0, 0);
      }
    }
    // B (weights, identical for every workgroup): LDS-DMA into buffer `buf`,
    // 64-byte rows [tap*NT + n]; chunk position p of row n holds k-chunk
    // p ^ ((n>>2)&3) (swizzle applied on the source address: LDS-DMA writes
    // lane-linear) so the ds_read_b128 column slices are conflict-free.
    const T* wb = reinterpret_cast<const T*>(a.w) + (int64_t)kdi * TAPS * a.cout_pad * a.cin_pad + c0;
    char* bdst = ldsB + buf * BBYTES;
#pragma unroll
    for (int jj = 0; jj < (NBI + 7) / 8; ++jj) {
      const int gi = wave + 8 * jj;
      if (gi < NBI) {
        const int row = gi * 16 + (lane >> 2);
        const int kc = (lane & 3) ^ ((row >> 2) & 3);
        const int tap = row / NT, nn = row - tap * NT;
        const T* src = wb + ((int64_t)tap * a.cout_pad + tl.n0 + nn) * a.cin_pad + kc * E;
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                         (void __attribute__((address_space(3)))*)(bdst + gi * 1024), 16, 0, 0);
      }
    }
  };
  auto commit = [&](int s) __attribute__((always_inline)) {
    const int c0 = (s % nchunk) * CK;
#pragma unroll
    for (int i = 0; i < MAXA; ++i) {
      const int q = tid + i * NTHR;
      if (q < SLOTS * 4) {
        const int c = c0 + (q & 3) * E;
        uint4 v = ra[i];
        if constexpr (VEC) v = mask_tail<T>(v, a.cin - c);
        if (a.prologue) v = prologue_lds<T>(v, c, relu_in, lsc, lsh);
        if (!((okmask >> i) & 1)) v = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(ldsA + (q >> 2) * ROWB + (q & 3) * 16) = v;
      }
    }
  };

  f32x16 acc[MS][NS];
#pragma unroll
  for (int m = 0; m < MS; ++m)
#pragma unroll
    for (int n = 0; n < NS; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;

  auto epilogue = [&](const Tile& tl) __attribute__((always_inline)) {
#pragma unroll
    for (int ms = 0; ms < MS; ++ms) {
      const int ho = tl.h0 + wave * MS + ms, wo = tl.w0 + r;
      if (ho < a.y.h && wo < a.y.w) {
#pragma unroll
        for (int ns = 0; ns < NS; ++ns) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int co = tl.n0 + ns * 32 + 8 * g + 4 * hf;
            if (co < a.cout) {
              const int valid = min(4, a.cout - co);
              float v[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                float t = acc[ms][ns][4 * g + e];
                if (a.bias && e < valid) {
                  int cb = co + e;
                  if (a.bias_r > 1) {  // view order (sub, c') -> torch order c'*r*r + sub
                    const int rr = a.bias_r * a.bias_r, cp = a.cout / rr;
                    const int sub = cb / cp;
                    cb = (cb - sub * cp) * rr + sub;
                  }
                  t += a.bias[cb];
                }
                t *= a.out_scale;
                if (a.act == VSRK_ACT_RELU) t = fmaxf(t, 0.f);
                v[e] = t;
              }
              const int64_t yo = view_off(a.y, tl.nb, tl.dz, ho, wo, co);
              const bool vec = (valid == 4) && ((yo & 3) == 0) &&
                               ((((uintptr_t)a.y.ptr) & (4 * sizeof(YT) - 1)) == 0);
              if (a.has_mask) {
                float m[4];
                load4<YT>(a.msk.ptr, view_off(a.msk, tl.nb, tl.dz, ho, wo, co), vec, valid, m);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = m[e] > 0.f ? v[e] : 0.f;
              }
              if (a.has_res) {
                float rr[4];
                load4<YT>(a.res.ptr, view_off(a.res, tl.nb, tl.dz, ho, wo, co), vec, valid, rr);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += rr[e];
              }
              if (a.accumulate) {
                float o[4];
                load4<YT>(a.y.ptr, yo, vec, valid, o);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += o[e];
              }
              YT* yp = reinterpret_cast<YT*>(a.y.ptr) + yo;
              if (vec) {
                if constexpr (sizeof(YT) == 4) {
                  *reinterpret_cast<float4*>(yp) = make_float4(v[0], v[1], v[2], v[3]);
                } else {
                  uint2 t;
                  bf16* b = reinterpret_cast<bf16*>(&t);
                  for (int e = 0; e < 4; ++e) b[e] = (bf16)v[e];
                  *reinterpret_cast<uint2*>(yp) = t;
                }
              } else {
                for (int e = 0; e < valid; ++e) yp[e] = from_f32<YT>(v[e]);
              }
            }
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MS; ++m)
#pragma unroll
      for (int n = 0; n < NS; ++n)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;
  };

  int t = t_lo + j;
  if (t >= t_hi) return;
  Tile cur = decode(t);
  int s = 0, buf = 0;
  issue(cur, 0, 0);
  if (a.prologue) __syncthreads();  // lsc/lsh visible before the first commit
  commit(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int xr = (r >> 2) & 3;  // B swizzle of this lane's rows
  const char* pa0 = ldsA + (wave * MS * HWd + r) * ROWB + hf * 16;
  while (true) {
    // next stage (possibly the first stage of the next tile)
    Tile nxt = cur;
    int ns_ = s + 1;
    bool have_next = true;
    if (ns_ >= cur.nst) {
      ns_ = 0;
      const int tn = t + gx;
      if (tn < t_hi) nxt = decode(tn); else have_next = false;
    }
    if (have_next) issue(nxt, ns_, buf ^ 1);
    const char* pb0 = ldsB + buf * BBYTES + r * 64;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int khi = 0; khi < KK; ++khi) {
#pragma unroll
        for (int kwi = 0; kwi < KK; ++kwi) {
          const int tap = khi * KK + kwi;
          uint4 bx[MS], aw[NS];
#pragma unroll
          for (int ms = 0; ms < MS; ++ms)
            bx[ms] = *reinterpret_cast<const uint4*>(pa0 + ((ms + khi) * HWd + kwi) * ROWB + ks * 32);
#pragma unroll
          for (int ns = 0; ns < NS; ++ns)
            aw[ns] = *reinterpret_cast<const uint4*>(pb0 + (tap * NT + ns * 32) * 64 + (((ks * 2 + hf) ^ xr) << 4));
#pragma unroll
          for (int ms = 0; ms < MS; ++ms)
#pragma unroll
            for (int ns = 0; ns < NS; ++ns) mma<T>(acc[ms][ns], aw[ns], bx[ms]);
        }
      }
    }
    if (s + 1 >= cur.nst) epilogue(cur);
    if (!have_next) break;
    __syncthreads();  // every wave is done reading A and B[buf]
    commit(ns_);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // B[buf^1] has landed
    __syncthreads();
    if (ns_ == 0) t += gx;
    cur = nxt;
    s = ns_;
    buf ^= 1;
  }
}

// ---------------------------------------------------------------------------
// weight packing
// ---------------------------------------------------------------------------
template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, T* __restrict__ out, int cout, int cin,
                                   int kd, int kh, int kw, int mode, int perm_r, int co_pad,
                                   int ci_pad, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  // out index = ((tap * co_pad + o) * ci_pad + i) in the packed (primed) roles
  const int i = idx % ci_pad;
  const int64_t t1 = idx / ci_pad;
  const int o = t1 % co_pad;
  const int tap = t1 / co_pad;
  const int kwi = tap % kw, khi = (tap / kw) % kh, kdi = tap / (kw * kh);
  int co, ci, sd, sh, sw;
  if (mode == 0) {
    co = o; ci = i; sd = kdi; sh = khi; sw = kwi;
  } else {
    co = i; ci = o; sd = kd - 1 - kdi; sh = kh - 1 - khi; sw = kw - 1 - kwi;
  }
  float v = 0.f;
  if (co < cout && ci < cin) {
    int cot = co;
    if (perm_r > 1) {  // view order (sub, c') -> torch order c'*r*r + sub
      const int rr = perm_r * perm_r, cp = cout / rr;
      const int sub = co / cp, cc = co - sub * cp;
      cot = cc * rr + sub;
    }
    v = w[((((int64_t)cot * cin + ci) * kd + sd) * kh + sh) * kw + sw];
  }
  out[idx] = from_f32<T>(v);
}

}  // namespace
extern "C" size_t vsrk_conv_packed_elems(int32_t cout, int32_t cin, int32_t kd, int32_t kh, int32_t kw,
                                         int32_t mode) {
  const int co = mode == 0 ? cout : cin, ci = mode == 0 ? cin : cout;
  return (size_t)kd * kh * kw * round_up(co, 128) * round_up(ci, 32);
}

extern "C" int vsrk_conv_pack_weight(int32_t dtype, const float* w, int32_t cout, int32_t cin, int32_t kd,
                                     int32_t kh, int32_t kw, int32_t mode, int32_t perm_r, void* packed,
                                     void* stream) {
  VSRK_CHECK(w && packed, "conv_pack_weight: null pointer");
  VSRK_CHECK(mode == 0 || mode == 1, "conv_pack_weight: mode must be 0 or 1");
  VSRK_CHECK(perm_r <= 1 || cout % (perm_r * perm_r) == 0, "conv_pack_weight: cout %% r^2 != 0");
  const int co = mode == 0 ? cout : cin, ci = mode == 0 ? cin : cout;
  const int co_pad = round_up(co, 128), ci_pad = round_up(ci, 32);
  const int64_t total = (int64_t)kd * kh * kw * co_pad * ci_pad;
  const int blk = 256;
  const int grid = (int)ceil_div64(total, blk);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VSRK_BF16)
    pack_weight_kernel<bf16><<<grid, blk, 0, s>>>(w, (bf16*)packed, cout, cin, kd, kh, kw, mode, perm_r,
                                                  co_pad, ci_pad, total);
  else
    pack_weight_kernel<float><<<grid, blk, 0, s>>>(w, (float*)packed, cout, cin, kd, kh, kw, mode, perm_r,
                                                   co_pad, ci_pad, total);
  VSRK_LAUNCH_CHECK("conv_pack_weight");
  return VSRK_OK;
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <typename T, int NT, int KK, bool VEC, typename YT>
static int launch_fwd(ConvArgs a, hipStream_t s) {
  constexpr int MS = NT >= 128 ? 1 : 2;  // rows per wave: keeps acc + staging under 256 VGPRs
  constexpr int FTH = 8 * MS;
  a.tiles_h = ceil_div(a.y.h, FTH);
  const int64_t ntiles = (int64_t)a.y.n * a.y.d * a.tiles_h * a.tiles_w * a.ntn;
  VSRK_CHECK(ntiles < (1ll << 31), "conv_fwd: too many tiles");
  a.ntiles = (int)ntiles;
  if (a.ntiles == 0) return VSRK_OK;
  const int slots = (FTH + KK - 1) * (TW + KK - 1);
  const size_t lds = (size_t)slots * ROWB + 2 * (size_t)KK * KK * NT * 64 + (a.prologue ? 2 * a.cin_pad * 4 : 0);
  auto kern = conv_fwd_kernel<T, NT, MS, KK, VEC, YT>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, NTHR, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const int64_t grid = std::min<int64_t>(ntiles, (int64_t)num_cus() * per_cu);
  a.nblk = (int)grid;
  kern<<<a.nblk, NTHR, lds, s>>>(a);
  VSRK_LAUNCH_CHECK("conv_fwd");
  return VSRK_OK;
}

template <typename T, int KK, bool VEC, typename YT>
static int dispatch_nt(const ConvArgs& a, int nt, hipStream_t s) {
  if (nt == 32) return launch_fwd<T, 32, KK, VEC, YT>(a, s);
  if (nt == 64) return launch_fwd<T, 64, KK, VEC, YT>(a, s);
  return launch_fwd<T, 128, KK, VEC, YT>(a, s);
}

template <typename T, typename YT>
static int dispatch_k(const ConvArgs& a, int nt, hipStream_t s) {
  if (a.kh == 1) return a.xvec ? dispatch_nt<T, 1, true, YT>(a, nt, s) : dispatch_nt<T, 1, false, YT>(a, nt, s);
  return a.xvec ? dispatch_nt<T, 3, true, YT>(a, nt, s) : dispatch_nt<T, 3, false, YT>(a, nt, s);
}

extern "C" int vsrk_conv_fwd(const vsrk_conv_desc* d, const vsrk_tensor5* x, const void* w_packed,
                             const float* bias, const float* pro_scale, const float* pro_shift,
                             const vsrk_tensor5* residual, const vsrk_tensor5* mask, const vsrk_tensor5* y,
                             void* stream) {
  VSRK_CHECK(d && x && y && w_packed, "conv_fwd: null argument");
  const int xdt = x->dtype, ydt = y->dtype;
  VSRK_CHECK(xdt == VSRK_F32 || xdt == VSRK_BF16, "conv_fwd: bad x dtype");
  VSRK_CHECK(ydt == xdt || ydt == VSRK_F32, "conv_fwd: y dtype must equal x dtype or be f32");
  const int es = xdt == VSRK_BF16 ? 2 : 4;
  if (!view_ok(x, "conv_fwd x") || !view_ok(y, "conv_fwd y")) return VSRK_ERR_INVALID;
  VSRK_CHECK(d->kh == d->kw && (d->kh == 1 || d->kh == 3) && d->kd >= 1,
             "conv_fwd: kernel %dx%dx%d unsupported (kh = kw in {1, 3})", d->kd, d->kh, d->kw);
  VSRK_CHECK(x->n == y->n, "conv_fwd: batch mismatch");
  VSRK_CHECK(x->h < 32768 && x->w < 32768, "conv_fwd: spatial size too large");
  VSRK_CHECK(!(d->prologue & VSRK_PRO_AFFINE) || (pro_scale && pro_shift), "conv_fwd: affine prologue needs scale/shift");
  const int yr = y->shuffle > 1 ? y->shuffle : 1;
  VSRK_CHECK(yr == 1 || (y->c / (yr * yr)) % 4 == 0, "conv_fwd: shuffled output needs c/r^2 %% 4 == 0");
  if (residual) {
    VSRK_CHECK(residual->dtype == ydt && residual->c == y->c && residual->h == y->h && residual->w == y->w,
               "conv_fwd: residual view mismatch");
  }
  if (mask) {
    VSRK_CHECK(mask->dtype == ydt && mask->c == y->c && mask->h == y->h && mask->w == y->w,
               "conv_fwd: mask view mismatch");
  }
  ConvArgs a;
  a.x = make_view(x);
  a.y = make_view(y);
  a.res = residual ? make_view(residual) : a.y;
  a.msk = mask ? make_view(mask) : a.y;
  a.w = (const char*)w_packed;
  a.bias = bias;
  a.pro_scale = pro_scale;
  a.pro_shift = pro_shift;
  a.cin = x->c;
  a.cout = y->c;
  a.cin_pad = round_up(x->c, 32);
  a.cout_pad = round_up(y->c, 128);
  a.kd = d->kd; a.kh = d->kh; a.kw = d->kw;
  a.pd = d->pd; a.ph = d->ph; a.pw = d->pw;
  a.prologue = d->prologue;
  a.act = d->act;
  a.accumulate = d->accumulate;
  a.has_res = residual != nullptr;
  a.has_mask = mask != nullptr;
  a.xvec = chunk_ok(x, es);
  a.bias_r = d->bias_perm_r;
  a.out_scale = d->out_scale;
  a.tiles_w = ceil_div(y->w, TW);
  // NT=128 only for 1x1 kernels (a double-buffered 3x3 weight slice of 128
  // channels would not fit LDS); wider 3x3 outputs use several 64-wide tiles
  const int NT = y->c <= 32 ? 32 : ((y->c <= 64 || d->kh == 3) ? 64 : 128);
  a.ntn = ceil_div(y->c, NT);
  hipStream_t s = (hipStream_t)stream;
  if (xdt == VSRK_BF16) {
    if (ydt == VSRK_BF16) return dispatch_k<bf16, bf16>(a, NT, s);
    return dispatch_k<bf16, float>(a, NT, s);
  }
  return dispatch_k<float, float>(a, NT, s);
}


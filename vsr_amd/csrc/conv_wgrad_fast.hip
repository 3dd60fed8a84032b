// Fast path of the weight/bias gradient (bf16 channels-last views, kh = kw in
// {1, 3}) on CDNA4: the autograd of nn.Conv2d/3d .weight/.bias in
// loss.backward() (base_trainer.py:128).  Same work decomposition, slab
// layout and deterministic reduce as conv_wgrad_kernel (conv_wgrad.hip):
// a workgroup owns a (32*NCO output x 32*NCI input channel, kd) combo and a
// run of 8 x 32-voxel tiles; its 4 waves (one per SIMD) own NCO x NCI channel
// blocks x NV voxel parts and run every kh*kw tap with
// v_mfma_f32_32x32x16_bf16 on ds_read_b64_tr_b16 (transposed) operands.
//
// Staging is the forward fast path's (conv_fast.hip):
//  * both operands (dY planes and the input halo planes, 64-byte rows of 32
//    channels) are staged by LDS-DMA, padding from a zero page; the lane ->
//    chunk roles and their element offsets are fixed per launch (a sub-pixel
//    view's sub-pixel is per channel plane, i.e. folded into the offsets);
//  * a two-slot ring, one barrier per tile: the next tile's DMA is issued
//    while this tile's MFMAs run, spread over its k-steps;
//  * fragments are software-pipelined one k-step ahead by hand;
//  * the optional BN-affine+ReLU prologue is applied by each lane to its own
//    landed input chunks, and dbias is summed by each lane over its own
//    landed dY chunks (both before the barrier that publishes the tile).
#include "conv_common.h"

namespace {
using namespace vsrk_conv;

__device__ __attribute__((aligned(256))) uint4 g_zero_page_w[16];

template <int NCO, int NCI, int KK>
struct WfGeom {
  static constexpr int PB = 64;               // plane row: 32 bf16 channels
  static constexpr int NV = 4 / (NCO * NCI);  // voxel parts
  static constexpr int VOX = GTH * TW;        // 256 voxels per tile
  static constexpr int VPW = VOX / NV;
  static constexpr int HWd = TW + KK - 1;
  static constexpr int SLOTS = (GTH + KK - 1) * HWd;
  static constexpr int SLOTP = (SLOTS + 15) / 16 * 16;
  static constexpr int TAPS = KK * KK;
  static constexpr int YI = NCO * VOX / 16;    // dY DMA wave-instructions per tile
  static constexpr int XI = NCI * SLOTP / 16;  // input DMA wave-instructions per tile
  static constexpr int YBYTES = NCO * VOX * PB;
  static constexpr int STAGE = YBYTES + NCI * SLOTP * PB;
  static constexpr int NYW = (YI + 3) / 4, NXW = (XI + 3) / 4;
  static constexpr int KSTEPS = VPW / 16;
  static constexpr int QPK = (NYW + NXW + KSTEPS - 1) / KSTEPS;  // DMA instructions per k-step
  static size_t lds_bytes(int prologue, int cin_pad) {
    const size_t red = (size_t)std::max(NCO * NCI * TAPS * 1024, GTHR * NYW * 8) * sizeof(float);
    return std::max((size_t)2 * STAGE + (prologue ? 2 * (size_t)cin_pad * 4 : 0), red);
  }
};

template <int NCO, int NCI, int KK, int PRO>
__global__ __attribute__((amdgpu_waves_per_eu(1, 1))) __launch_bounds__(GTHR) void conv_wgrad_fast_kernel(
    WgradArgs a) {
  using G = WfGeom<NCO, NCI, KK>;
  constexpr int PB = G::PB, NV = G::NV, VOX = G::VOX, VPW = G::VPW, HWd = G::HWd, SLOTS = G::SLOTS,
                SLOTP = G::SLOTP, TAPS = G::TAPS, YI = G::YI, XI = G::XI, YBYTES = G::YBYTES, STAGE = G::STAGE,
                NYW = G::NYW, NXW = G::NXW, KSTEPS = G::KSTEPS, QPK = G::QPK;
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cis = wave % NCI, cos_ = (wave / NCI) % NCO, vp = wave / (NCI * NCO);
  float* lsc = reinterpret_cast<float*>(lds + 2 * STAGE);
  float* lsh = lsc + a.cin_pad;

  const int L = xcd_remap(blockIdx.x, a.nblk);
  const int split = L / a.ncombos;
  int combo = L - split * a.ncombos;
  const int cot = combo % a.n_co_tiles;
  combo /= a.n_co_tiles;
  const int cic = combo % a.n_ci_chunks;
  const int kdi = combo / a.n_ci_chunks;
  const int co0 = cot * 32 * NCO, ci0 = cic * 32 * NCI;
  const bool do_bias = a.want_bias && cic == 0 && kdi == a.kd_bias;
  if constexpr (PRO) {
    stage_prologue(lsc, lsh, a.prologue, a.pro_scale, a.pro_shift, a.cin, a.cin_pad, tid, GTHR);
    __syncthreads();
  }
  const bool relu_in = (a.prologue & VSRK_PRO_RELU) != 0;

  // ---- fixed DMA roles: instruction i = wave + 4k; lane -> row lane/4, piece lane%4
  const int yr = a.dy.r, xr = a.x.r;
  int y_rel[NYW], y_geo[NYW], y_ch[NYW];
#pragma unroll
  for (int k = 0; k < NYW; ++k) {
    const int i = wave + 4 * k;
    const int pl = i / (VOX / 16);
    const int v = (i % (VOX / 16)) * 16 + (lane >> 2);
    const int row = v / TW, col = v % TW;
    const int ch = co0 + pl * 32 + 8 * (lane & 3);
    int sub = 0, cc = ch;
    if (yr > 1) {
      sub = ch / a.dy.cphys;
      cc = ch - sub * a.dy.cphys;
    }
    y_rel[k] = (int)((int64_t)(row * yr + sub / yr) * a.dy.sh + (int64_t)(col * yr + sub % yr) * a.dy.sw) + cc;
    y_geo[k] = i < YI ? ((row << 8) | col) : -1;
    y_ch[k] = ch;
  }
  int x_rel[NXW], x_geo[NXW], x_ch[NXW];
#pragma unroll
  for (int k = 0; k < NXW; ++k) {
    const int i = wave + 4 * k;
    const int pl = i / (SLOTP / 16);
    const int s = (i % (SLOTP / 16)) * 16 + (lane >> 2);
    const int hh = s / HWd, ww = s % HWd;
    const int ch = ci0 + pl * 32 + 8 * (lane & 3);
    int sub = 0, cc = ch;
    if (xr > 1) {
      sub = ch / a.x.cphys;
      cc = ch - sub * a.x.cphys;
    }
    x_rel[k] = (int)((int64_t)(hh * xr + sub / xr) * a.x.sh + (int64_t)(ww * xr + sub % xr) * a.x.sw) + cc;
    x_geo[k] = (i < XI && s < SLOTS) ? ((hh << 8) | ww) : -1;
    x_ch[k] = ch;
  }

  const char* zp = reinterpret_cast<const char*>(g_zero_page_w);
  struct Dma {
    const bf16* yb;
    const bf16* xb;
    uint32_t sbase;
    unsigned ym, xm;
    bool on;
  };
  auto tile_ok = [&](int t) __attribute__((always_inline)) {
    const int dz = (t / (a.tiles_w * a.tiles_h)) % a.dy.d;
    const int di = dz + kdi - a.pd;
    return di >= 0 && di < a.x.d;
  };
  auto prep = [&](int t, int slot) __attribute__((always_inline)) {
    Dma d;
    int b = t;
    const int tw_i = b % a.tiles_w;
    b /= a.tiles_w;
    const int th_i = b % a.tiles_h;
    b /= a.tiles_h;
    const int dz = b % a.dy.d;
    const int nb = b / a.dy.d;
    const int h0 = th_i * GTH, w0 = tw_i * TW;
    const int di = dz + kdi - a.pd;
    const int hb = h0 - a.ph, wb = w0 - a.pw;
    d.yb = reinterpret_cast<const bf16*>(a.dy.ptr) +
           (nb * a.dy.sn + (int64_t)dz * a.dy.sd + (int64_t)h0 * yr * a.dy.sh + (int64_t)w0 * yr * a.dy.sw);
    d.xb = reinterpret_cast<const bf16*>(a.x.ptr) +
           (nb * a.x.sn + (int64_t)di * a.x.sd + (int64_t)hb * xr * a.x.sh + (int64_t)wb * xr * a.x.sw);
    d.ym = 0;
#pragma unroll
    for (int k = 0; k < NYW; ++k) {
      const int row = y_geo[k] >> 8, col = y_geo[k] & 0xff;
      const bool ok = y_geo[k] >= 0 && h0 + row < a.dy.h && w0 + col < a.dy.w && y_ch[k] < a.cout;
      d.ym |= (ok ? 1u : 0u) << k;
    }
    d.xm = 0;
#pragma unroll
    for (int k = 0; k < NXW; ++k) {
      const int hh = x_geo[k] >> 8, ww = x_geo[k] & 0xff;
      const bool ok = x_geo[k] >= 0 && hb + hh >= 0 && hb + hh < a.x.h && wb + ww >= 0 && wb + ww < a.x.w &&
                      x_ch[k] < a.cin;
      d.xm |= (ok ? 1u : 0u) << k;
    }
    d.sbase = lds_addr(lds) + slot * STAGE;
    d.on = true;
    return d;
  };
  auto dma = [&](const Dma& d, int q) __attribute__((always_inline)) {
    if (q < NYW) {
      const int i = wave + 4 * q;
      if (i < YI) {
        const void* src = ((d.ym >> q) & 1) ? (const void*)(d.yb + y_rel[q]) : (const void*)zp;
        glds16(src, d.sbase + i * 1024);
      }
    } else if (q < NYW + NXW) {
      const int k = q - NYW, i = wave + 4 * k;
      if (i < XI) {
        const void* src = ((d.xm >> k) & 1) ? (const void*)(d.xb + x_rel[k]) : (const void*)zp;
        glds16(src, d.sbase + YBYTES + i * 1024);
      }
    }
  };

  f32x16 acc[TAPS];
#pragma unroll
  for (int t = 0; t < TAPS; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  float bsum[NYW][8];
#pragma unroll
  for (int k = 0; k < NYW; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) bsum[k][e] = 0.f;

  // after this lane's own DMA landed: prologue on its input chunks, dbias over its dY chunks
  auto own_pass = [&](int slot, const Dma& d) __attribute__((always_inline)) {
    if constexpr (PRO) {
#pragma unroll
      for (int k = 0; k < NXW; ++k) {
        const int i = wave + 4 * k;
        if (i < XI && ((d.xm >> k) & 1)) {
          uint4* p = reinterpret_cast<uint4*>(lds + slot * STAGE + YBYTES + i * 1024 + lane * 16);
          *p = prologue_lds<bf16>(*p, x_ch[k], relu_in, lsc, lsh);
        }
      }
    }
    if (do_bias) {
#pragma unroll
      for (int k = 0; k < NYW; ++k) {
        const int i = wave + 4 * k;
        if (i < YI && ((d.ym >> k) & 1)) {
          float f[8];
          Chunk<bf16>::unpack(*reinterpret_cast<const uint4*>(lds + slot * STAGE + i * 1024 + lane * 16), f);
#pragma unroll
          for (int e = 0; e < 8; ++e) bsum[k][e] += f[e];
        }
      }
    }
  };

  // transposed fragment reads (as conv_wgrad_kernel): group g = lane>>4 reads a
  // 4-row x 16-column block; lane 4q+p addresses row q, columns 4p..4p+3.
  const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
  const int hfk = g >> 1, colb = ((g & 1) * 16 + 4 * pp) * 2;
  struct Frags {
    v4i16 y0, y1, x0[TAPS], x1[TAPS];
  };
  auto compute = [&](int slot, const Dma& d) __attribute__((always_inline)) {
    const char* py = lds + slot * STAGE + cos_ * VOX * PB;
    const char* px = lds + slot * STAGE + YBYTES + cis * SLOTP * PB;
    auto load = [&](Frags& f, int ks) __attribute__((always_inline)) {
      const int vb = vp * VPW + ks * 16;
      const int vrow = vb / TW, vcol0 = (vb % TW) + 8 * hfk;
      f.y0 = ds_read_tr(py + (vrow * TW + vcol0 + qq) * PB + colb);
      f.y1 = ds_read_tr(py + (vrow * TW + vcol0 + 4 + qq) * PB + colb);
#pragma unroll
      for (int kh = 0; kh < KK; ++kh)
#pragma unroll
        for (int kw = 0; kw < KK; ++kw) {
          const char* xs = px + ((vrow + kh) * HWd + vcol0 + kw + qq) * PB + colb;
          f.x0[kh * KK + kw] = ds_read_tr(xs);
          f.x1[kh * KK + kw] = ds_read_tr(xs + 4 * PB);
        }
    };
    Frags fr[2];
    load(fr[0], 0);
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      if (ks + 1 < KSTEPS) load(fr[(ks + 1) & 1], ks + 1);
      const Frags& f = fr[ks & 1];
      const bf16x8 af = __builtin_bit_cast(bf16x8, __builtin_shufflevector(f.y0, f.y1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int tp = 0; tp < TAPS; ++tp) {
        const bf16x8 bfr =
            __builtin_bit_cast(bf16x8, __builtin_shufflevector(f.x0[tp], f.x1[tp], 0, 1, 2, 3, 4, 5, 6, 7));
        acc[tp] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc[tp], 0, 0, 0);
      }
      if (d.on) {
#pragma unroll
        for (int q = ks * QPK; q < (ks + 1) * QPK; ++q) dma(d, q);
      }
    }
  };

  const int t_begin = split * a.tiles_per_split;
  const int t_end = min(a.ntiles, t_begin + a.tiles_per_split);
  int t = t_begin;
  while (t < t_end && !tile_ok(t)) ++t;
  if (t < t_end) {
    int slot = 0;
    Dma dc = prep(t, 0);
#pragma unroll
    for (int q = 0; q < NYW + NXW; ++q) dma(dc, q);
    while (true) {
      int tn = t + 1;
      while (tn < t_end && !tile_ok(tn)) ++tn;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile t landed
      own_pass(slot, dc);
      __syncthreads();  // every wave's DMA (and prologue) of tile t visible; slot^1 free
      Dma dn;
      dn.on = false;
      if (tn < t_end) dn = prep(tn, slot ^ 1);
      compute(slot, dn);
      if (tn >= t_end) break;
      t = tn;
      slot ^= 1;
      dc = dn;
    }
  }

  // slab layout: [tap][co (32*NCO)][ci (32*NCI)] then dbias[32*NCO]
  float* out = a.ws + (int64_t)L * a.slab;
  constexpr int NW = TAPS * 1024 * NCO * NCI;
  const int r = lane & 31, hfo = lane >> 5;
  if constexpr (NV == 1) {
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int co = cos_ * 32 + (i & 3) + 8 * (i >> 2) + 4 * hfo;
        out[(tap * 32 * NCO + co) * (32 * NCI) + cis * 32 + r] = acc[tap][i];
      }
    }
  } else {
    // fixed-order sum of the NV voxel-part partials: red[cos][cis][tap][co][ci]
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);
    for (int v = 0; v < NV; ++v) {
      if (vp == v) {
#pragma unroll
        for (int tap = 0; tap < TAPS; ++tap) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int co = (i & 3) + 8 * (i >> 2) + 4 * hfo;
            float* dst = red + (((cos_ * NCI + cis) * TAPS + tap) * 32 + co) * 32 + r;
            *dst = (v == 0) ? acc[tap][i] : *dst + acc[tap][i];
          }
        }
      }
      __syncthreads();
    }
    for (int i = tid; i < NW; i += GTHR) {
      const int ci = i % (32 * NCI);
      const int t2 = i / (32 * NCI);
      const int co = t2 % (32 * NCO);
      const int tap = t2 / (32 * NCO);
      out[i] = red[((((co / 32) * NCI + ci / 32) * TAPS + tap) * 32 + (co % 32)) * 32 + (ci % 32)];
    }
  }
  if (do_bias) {
    // partials of lane (wave, k) cover channels y_ch[k] - co0 .. +7; summed in a fixed order
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int k = 0; k < NYW; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(tid * NYW + k) * 8 + e] = bsum[k][e];
    __syncthreads();
    if (tid < 32 * NCO) {
      const int c = tid;  // channel within the combo's 32*NCO block
      const int pl = c / 32, piece = (c % 32) / 8, e = c % 8;
      float sacc = 0.f;
      // instruction i carries plane i / (VOX/16); lanes with (lane & 3) == piece hold channel c
      for (int i = pl * (VOX / 16); i < (pl + 1) * (VOX / 16); ++i) {
        const int w_ = i % 4, k = i / 4;
        for (int ln = piece; ln < 64; ln += 4) sacc += red[((w_ * 64 + ln) * NYW + k) * 8 + e];
      }
      out[NW + c] = sacc;
    }
  }
}

template <int NCO, int NCI, int KK>
bool launch_wgrad_fast(const WgradArgs& a, hipStream_t s) {
  const size_t lds = WfGeom<NCO, NCI, KK>::lds_bytes(a.prologue, a.cin_pad);
  if (lds > 160 * 1024) return false;
  if (a.prologue) {
    auto kern = conv_wgrad_fast_kernel<NCO, NCI, KK, 1>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<a.nblk, GTHR, lds, s>>>(a);
  } else {
    auto kern = conv_wgrad_fast_kernel<NCO, NCI, KK, 0>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<a.nblk, GTHR, lds, s>>>(a);
  }
  return true;
}

template <int NCO, int NCI>
bool wgrad_fast_k(const WgradArgs& a, hipStream_t s) {
  return a.kh == 3 ? launch_wgrad_fast<NCO, NCI, 3>(a, s) : launch_wgrad_fast<NCO, NCI, 1>(a, s);
}

}  // namespace

// 1 = launched; 0 = not eligible (the generic kernel runs).  Needs bf16
// chunk-readable views (checked by the caller), kh = kw in {1, 3}, channel
// counts in whole 16-byte chunks and sub-pixel planes of whole 32-channel rows.
int vsrk_g_wgrad_fast_mode = -1;  // -1: from VSRK_WGRAD_FAST (default off), 0 off, 1 on (vsrk_conv_set_path)

int vsrk_conv_wgrad_fast(const vsrk_conv::WgradArgs& a, int nco, int nci, hipStream_t s) {
  int mode = vsrk_g_wgrad_fast_mode;
  if (mode < 0) {
    // opt-in: at one workgroup of 4 waves per CU it trails conv_wgrad_kernel
    // (2 workgroups per CU) on the EDSR 64->64 shape
    const char* e = getenv("VSRK_WGRAD_FAST");
    mode = (e && e[0] == '1') ? 1 : 0;
  }
  if (!mode) return 0;
  if (a.kh != a.kw || (a.kh != 1 && a.kh != 3)) return 0;
  if (a.cin % 8 || a.cout % 8) return 0;
  if (a.x.r > 1 && a.x.cphys % 32) return 0;
  if (a.dy.r > 1 && a.dy.cphys % 32) return 0;
  bool ok;
  if (nco == 2 && nci == 2) ok = wgrad_fast_k<2, 2>(a, s);
  else if (nco == 2) ok = wgrad_fast_k<2, 1>(a, s);
  else if (nci == 2) ok = wgrad_fast_k<1, 2>(a, s);
  else ok = wgrad_fast_k<1, 1>(a, s);
  return ok ? 1 : 0;
}

// Pipelined 3x3(x3) weight/bias gradient for 16-bit channels-last views: the
// autograd of nn.Conv2d/Conv3d(k=3).weight/.bias in loss.backward()
// (base_trainer.py:128; duf_net.py:203,214 and edsr_net.py:28-64 are the
// convs it serves).  Same work decomposition, slab layout and deterministic
// reduce as conv_wgrad_kernel (conv_wgrad.hip): a workgroup owns a
// (32*NCO output x 32*NCI input channel, kd) combo and a run of 8 x 32-voxel
// tiles; its 4 waves (one per SIMD) own NCO x NCI channel blocks x NV voxel
// parts and run the nine (kh, kw) taps with v_mfma_f32_32x32x16_{bf16,f16} on
// ds_read_b64_tr_b16 operands.
//
// What differs is the staging, which is what bounded the generic kernel
// (PMC on the DUF 64->32 3x3x3 wgrad with the BN+ReLU prologue: 17 VALU and
// 4 SALU per MFMA, MFMA busy 22 %):
//  * a two-stage LDS ring with ONE barrier per tile: tile t+1 is written into
//    the other stage while tile t's MFMAs run, chunk by chunk between the
//    k-steps, so the prologue's VALU fills MFMA gaps instead of a serial phase;
//  * loads run two tiles ahead: each register chunk is refilled (tile t+2)
//    right after it is committed (tile t+1);
//  * raw buffer loads with launch-fixed per-thread byte offsets: per tile a
//    chunk costs an add, two range compares and a select (out-of-range ->
//    an offset past the buffer, which reads as zero: the conv's zero padding);
//  * the prologue's per-channel scale/shift live in registers (every thread
//    stages one fixed 8-channel chunk position), the ReLU is compile-time and
//    16-bit packing is v_cvt_pk_{bf16,f16}_f32 on vector converts.
#include "conv_common.h"


namespace {
using namespace vsrk_conv;

typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr uint32_t OOB = 0x80000000u;
__device__ __forceinline__ Rsrc rsrc_at(const void* base) {
  const uint64_t b = (uint64_t)base;
  const uint64_t u = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, 0, 0x7FFFFFF0, 0x00020000);
}
__device__ __forceinline__ uint4 bload16(Rsrc r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

// 2 packed 16-bit values <-> 2 floats
template <typename T> __device__ __forceinline__ f32x2_t unpack2(uint32_t v);
template <> __device__ __forceinline__ f32x2_t unpack2<bf16>(uint32_t v) {
  return f32x2_t{__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)};
}
template <> __device__ __forceinline__ f32x2_t unpack2<f16>(uint32_t v) {
  return __builtin_convertvector(__builtin_bit_cast(f16x2_t, v), f32x2_t);
}
template <typename T> __device__ __forceinline__ uint32_t pack2(f32x2_t f);
template <> __device__ __forceinline__ uint32_t pack2<bf16>(f32x2_t f) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_t));
}
template <> __device__ __forceinline__ uint32_t pack2<f16>(f32x2_t f) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, f16x2_t));
}

// BN-affine (+ReLU) of one 8-channel chunk with the channel constants in registers
template <typename T, int PRO>
__device__ __forceinline__ uint4 pro8(uint4 v, const f32x2_t* sc, const f32x2_t* sh) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x2_t f = unpack2<T>(w[i]);
    if constexpr (PRO & VSRK_PRO_AFFINE) f = f * sc[i] + sh[i];
    if constexpr (PRO & VSRK_PRO_RELU) {
      f.x = fmaxf(f.x, 0.f);
      f.y = fmaxf(f.y, 0.f);
    }
    w[i] = pack2<T>(f);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <int NCO, int NCI>
struct WpGeom {
  static constexpr int KK = 3;
  static constexpr int PB = 64;                // plane row: 32 16-bit channels
  static constexpr int NV = 4 / (NCO * NCI);   // voxel parts
  static constexpr int VOX = GTH * TW;         // 256 voxels per tile
  static constexpr int VPW = VOX / NV;
  static constexpr int KSTEPS = VPW / 16;
  static constexpr int HWd = TW + KK - 1;      // 34
  static constexpr int SLOTS = (GTH + KK - 1) * HWd;  // 340
  static constexpr int TAPS = KK * KK;
  static constexpr int YCPV = NCO * 4;         // dY chunks per voxel
  static constexpr int XCPV = NCI * 4;         // X chunks per slot
  static constexpr int MAXY = VOX * YCPV / GTHR;
  static constexpr int MAXX = (SLOTS * XCPV + GTHR - 1) / GTHR;
  static constexpr int NCH = MAXY + MAXX;      // chunks per thread per tile
  static constexpr int XSSTEP = GTHR / XCPV;   // slot stride between a thread's X chunks
  static constexpr int SLOTP = MAXX * XSSTEP;  // padded slots: every chunk role has a home (no branch)
  // channel-block planes padded by 64 B: the two planes an 8-lane group of a
  // commit's ds_write_b128 touches (lanes 0-3 block 0, 4-7 block 1) would
  // otherwise start on the same bank (plane sizes are multiples of 256 B):
  // 26 % of LDS cycles were bank conflicts (PMC, EDSR 64->64 wgrad)
  static constexpr int YPL = VOX * PB + 64;
  static constexpr int XPL = SLOTP * PB + 64;
  static constexpr int YBYTES = NCO * YPL;
  static constexpr int STAGE = YBYTES + NCI * XPL;
  static size_t lds_bytes() {
    const size_t red = NV > 1 ? (size_t)NCO * NCI * TAPS * 1024 * sizeof(float) : 0;
    const size_t bias = (size_t)GTHR * 8 * sizeof(float);
    return std::max((size_t)2 * STAGE, std::max(red, bias));
  }
};

// ABL (A/B builds only, VSRK_WP_EXP): 1 = no staging inside the tile loop,
// 2 = no fragment reads / MFMAs (the ceilings of either half)
template <typename T, int NCO, int NCI, int PRO, int ABL>
__global__ __attribute__((amdgpu_waves_per_eu(1, 1))) __launch_bounds__(GTHR) void conv_wgrad_pipe_kernel(
    WgradArgs a) {
  using G = WpGeom<NCO, NCI>;
  constexpr int KK = G::KK, PB = G::PB, NV = G::NV, VOX = G::VOX, VPW = G::VPW, KSTEPS = G::KSTEPS,
                HWd = G::HWd, SLOTS = G::SLOTS, TAPS = G::TAPS, YCPV = G::YCPV, XCPV = G::XCPV, MAXY = G::MAXY,
                MAXX = G::MAXX, NCH = G::NCH, YBYTES = G::YBYTES, STAGE = G::STAGE, SLOTP = G::SLOTP;
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cis = wave % NCI, cos_ = (wave / NCI) % NCO, vp = wave / (NCI * NCO);

  const int L = xcd_remap(blockIdx.x, a.nblk);
  const int split = L / a.ncombos;
  int combo = L - split * a.ncombos;
  const int cot = combo % a.n_co_tiles;
  combo /= a.n_co_tiles;
  const int cic = combo % a.n_ci_chunks;
  const int kdi = combo / a.n_ci_chunks;
  const int co0 = cot * 32 * NCO, ci0 = cic * 32 * NCI;
  const bool do_bias = a.want_bias && cic == 0 && kdi == a.kd_bias;
  // taps of this wave's channel block pair that carry a weight (sub-pixel
  // forms: DRF's projections, 4 of 9; the rest stay zero in the slab)
  const unsigned tmk = a.sp_by == 1 ? a.sptap[(co0 >> 5) + cos_] : (a.sp_by == 2 ? a.sptap[(ci0 >> 5) + cis] : 0x1ffu);

  // ---- launch-fixed per-thread chunk roles ----
  const int yrem = tid % YCPV, xrem = tid % XCPV;
  const int yc = co0 + (yrem >> 2) * 32 + (yrem & 3) * 8;
  const int xc = ci0 + (xrem >> 2) * 32 + (xrem & 3) * 8;
  const bool yc_ok = yc < a.cout, xc_ok = xc < a.cin;
  const int ydst = (yrem >> 2) * G::YPL + (yrem & 3) * 16;
  const int xdst = (xrem >> 2) * G::XPL + (xrem & 3) * 16;
  const int ybase_vox = tid / YCPV, xbase_slot = tid / XCPV;
  constexpr int YVSTEP = GTHR / YCPV, XSSTEP = G::XSSTEP;
  // byte offsets within an (n, d) slice, relative to the tile origin.  A
  // sub-pixel view (r > 1) keeps logical channel c = (i*r + j)*cphys + c' at
  // physical (h*r + i, w*r + j, c'): an 8-channel chunk never straddles
  // sub-pixels (cphys % 8 == 0), so (i, j, c') is a per-thread constant.
  const int ysh = (int)a.dy.sh * 2, ysw = (int)a.dy.sw * 2;
  const int xsh = (int)a.x.sh * 2, xsw = (int)a.x.sw * 2;
  auto chan_off = [](const View& v, int c, int sh2, int sw2) {
    if (v.r == 1) return c * 2;
    const int sub = c / v.cphys, cc = c - sub * v.cphys;
    const int i = sub / v.r, j = sub - i * v.r;
    return i * sh2 + j * sw2 + cc * 2;
  };
  const int ycoff = chan_off(a.dy, yc_ok ? yc : 0, ysh, ysw), xcoff = chan_off(a.x, xc_ok ? xc : 0, xsh, xsw);
  const int ysh_r = ysh * a.dy.r, ysw_r = ysw * a.dy.r, xsh_r = xsh * a.x.r, xsw_r = xsw * a.x.r;
  uint32_t yrel[MAXY], xrel[MAXX];
#pragma unroll
  for (int i = 0; i < MAXY; ++i) {
    const int v = ybase_vox + i * YVSTEP;
    yrel[i] = (uint32_t)((v / TW) * ysh_r + (v % TW) * ysw_r + ycoff);
  }
#pragma unroll
  for (int i = 0; i < MAXX; ++i) {
    const int s = xbase_slot + i * XSSTEP;
    xrel[i] = (uint32_t)((s / HWd) * xsh_r + (s % HWd) * xsw_r + xcoff);
  }

  // prologue constants of this thread's 8 input channels
  f32x2_t psc[4], psh[4];
  if constexpr (PRO & VSRK_PRO_AFFINE) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = xc + 2 * i;
      psc[i] = f32x2_t{c < a.cin ? a.pro_scale[c] : 0.f, c + 1 < a.cin ? a.pro_scale[c + 1] : 0.f};
      psh[i] = f32x2_t{c < a.cin ? a.pro_shift[c] : 0.f, c + 1 < a.cin ? a.pro_shift[c + 1] : 0.f};
    }
  }

  // ---- tile walk (valid tiles only: the depth tap must land inside x) ----
  const int t_begin = split * a.tiles_per_split;
  const int t_end = min(a.ntiles, t_begin + a.tiles_per_split);
  // a scalar cursor (tile index and its decoded coordinates) advanced with
  // carries: no divisions per tile
  struct Cur {
    int t, tw, th, dz, nb;
  };
  auto decode = [&](int t) __attribute__((always_inline)) {
    Cur c;
    c.t = t;
    c.tw = t % a.tiles_w;
    t /= a.tiles_w;
    c.th = t % a.tiles_h;
    t /= a.tiles_h;
    c.dz = t % a.dy.d;
    c.nb = t / a.dy.d;
    return c;
  };
  auto next_slab = [&](Cur& c) __attribute__((always_inline)) {
    c.tw = 0;
    c.th = 0;
    if (++c.dz == a.dy.d) {
      c.dz = 0;
      ++c.nb;
    }
  };
  // the first valid tile at or after c (the depth tap must land inside x)
  auto skip_invalid = [&](Cur& c) __attribute__((always_inline)) {
    while (c.t < t_end) {
      const int di = c.dz + kdi - a.pd;
      if (di >= 0 && di < a.x.d) break;
      c.t += (a.tiles_w - c.tw) + (a.tiles_h - 1 - c.th) * a.tiles_w;
      next_slab(c);
    }
  };
  auto advance = [&](Cur& c) __attribute__((always_inline)) {
    if (c.t >= t_end) return;
    ++c.t;
    if (++c.tw == a.tiles_w) {
      c.tw = 0;
      if (++c.th == a.tiles_h) {
        c.th = 0;
        if (++c.dz == a.dy.d) {
          c.dz = 0;
          ++c.nb;
        }
      }
    }
    skip_invalid(c);
  };

  // per-tile scalar state of an in-flight load set
  struct TileRefs {
    Rsrc ry, rx;
    int h0, w0;  // dY origin; x origin is (h0 - ph, w0 - pw)
  };
  auto tile_refs = [&](const Cur& c) __attribute__((always_inline)) {
    TileRefs r;
    const int di = c.dz + kdi - a.pd;
    r.h0 = c.th * GTH;
    r.w0 = c.tw * TW;
    const char* yb = a.dy.ptr + ((int64_t)c.nb * a.dy.sn + (int64_t)c.dz * a.dy.sd) * 2 +
                     ((int64_t)r.h0 * a.dy.sh + (int64_t)r.w0 * a.dy.sw) * 2 * a.dy.r;
    const char* xb = a.x.ptr + ((int64_t)c.nb * a.x.sn + (int64_t)di * a.x.sd) * 2 +
                     ((int64_t)(r.h0 - a.ph) * a.x.sh + (int64_t)(r.w0 - a.pw) * a.x.sw) * 2 * a.x.r;
    r.ry = rsrc_at(yb);
    r.rx = rsrc_at(xb);
    return r;
  };
  // chunk i of a tile: i < MAXY are dY chunks, the rest X chunks.  `live` =
  // the tile exists (else the chunk reads as zero).  X chunks record their
  // in-range bit in xm (the prologue's output is re-zeroed where it is off).
  uint32_t xm = 0;
  auto load_chunk = [&](int i, const TileRefs& r, bool live) __attribute__((always_inline)) -> uint4 {
    if (i < MAXY) {
      const int v = ybase_vox + i * YVSTEP;
      const bool ok = live & yc_ok & ((unsigned)(r.h0 + v / TW) < (unsigned)a.dy.h) &
                      ((unsigned)(r.w0 + v % TW) < (unsigned)a.dy.w);
      return bload16(r.ry, ok ? yrel[i] : OOB);
    } else {
      const int j = i - MAXY;
      const int s = xbase_slot + j * XSSTEP;
      const bool ok = live & xc_ok & (s < SLOTS) & ((unsigned)(r.h0 - a.ph + s / HWd) < (unsigned)a.x.h) &
                      ((unsigned)(r.w0 - a.pw + s % HWd) < (unsigned)a.x.w);
      xm = (xm & ~(1u << j)) | ((ok ? 1u : 0u) << j);
      return bload16(r.rx, ok ? xrel[j] : OOB);
    }
  };
  float bsum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bsum[e] = 0.f;
  auto commit_y = [&](int i, uint4 v, char* stage) __attribute__((always_inline)) {
    const int v_ = ybase_vox + i * YVSTEP;
    *reinterpret_cast<uint4*>(stage + ydst + v_ * PB) = v;
    if (do_bias) {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x2_t f = unpack2<T>(w[q]);
        bsum[2 * q] += f.x;
        bsum[2 * q + 1] += f.y;
      }
    }
  };
  // branch-free: slots past SLOTS land in the padding of the stage
  auto commit_x = [&](int j, uint4 v, char* stage) __attribute__((always_inline)) {
    const int s = xbase_slot + j * XSSTEP;
    if constexpr (PRO != 0) {
      // the conv pads the *activated* input with zeros
      v = pro8<T, PRO>(v, psc, psh);
      const bool ok = (xm >> j) & 1u;
      v.x = ok ? v.x : 0u;
      v.y = ok ? v.y : 0u;
      v.z = ok ? v.z : 0u;
      v.w = ok ? v.w : 0u;
    }
    *reinterpret_cast<uint4*>(stage + YBYTES + xdst + s * PB) = v;
  };

  f32x16 acc[TAPS];
#pragma unroll
  for (int t = 0; t < TAPS; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  uint4 rg[NCH];
  Cur c0 = decode(t_begin);
  skip_invalid(c0);
  const Cur cfirst = c0;  // a valid address for the dead loads past the end
  {
    const TileRefs r0 = tile_refs(c0.t < t_end ? c0 : cfirst);
#pragma unroll
    for (int i = 0; i < NCH; ++i) rg[i] = load_chunk(i, r0, c0.t < t_end);
#pragma unroll
    for (int i = 0; i < MAXY; ++i) commit_y(i, rg[i], lds);
#pragma unroll
    for (int j = 0; j < MAXX; ++j) commit_x(j, rg[MAXY + j], lds);
  }
  Cur c1 = c0;
  advance(c1);
  TileRefs rn = tile_refs(c1.t < t_end ? c1 : cfirst);
#pragma unroll
  for (int i = 0; i < NCH; ++i) rg[i] = load_chunk(i, rn, c1.t < t_end);
  __syncthreads();

  int stage_i = 0;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  const int hfk = g >> 1, colb = ((g & 1) * 16 + 4 * p) * 2;
  constexpr int ROWS = VPW / TW;           // dY rows of a wave's voxel part
  constexpr int NSTEP = (ROWS + KK - 1) * 2;  // (input row, half) steps per tile
  const int vr0 = vp * ROWS;
  while (c0.t < t_end) {
    const char* cur = lds + stage_i * STAGE;
    char* nxt = lds + (stage_i ^ 1) * STAGE;
    Cur c2 = c1;
    advance(c2);
    const bool have_nn = c2.t < t_end;
    const TileRefs rnn = tile_refs(have_nn ? c2 : cfirst);
    const char* py = cur + cos_ * G::YPL;
    const char* px = cur + YBYTES + cis * G::XPL;
    // Row-reuse walk: a wave holds the dY fragments of its ROWS rows (both
    // 16-voxel halves) and walks the XR = ROWS + 2 input rows once; each
    // input fragment (row xr, half c, tap kw) serves every kh with dY row
    // xr - kh inside the wave's rows.  Per accumulator the MFMA order is
    // still (dY row, half) ascending, as in conv_wgrad_kernel.
    uint4 fa[ROWS][2];
    if constexpr (!(ABL & 2)) {
#pragma unroll
      for (int r = 0; r < ROWS; ++r)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const char* ys = py + ((vr0 + r) * TW + c * 16 + 8 * hfk + q) * PB + colb;
          const v4i16 y0 = ds_read_tr(ys);
          const v4i16 y1 = ds_read_tr(ys + 4 * PB);
          fa[r][c] = __builtin_bit_cast(uint4, __builtin_shufflevector(y0, y1, 0, 1, 2, 3, 4, 5, 6, 7));
        }
    }
    // input fragments are software-pipelined one step ahead: the reads of
    // step st + 1 are issued (fenced from the scheduler) before step st's
    // MFMAs, which consume the reads issued one step earlier
    auto read_b = [&](int st, uint4* fb) __attribute__((always_inline)) {
      const int xr = st >> 1, c = st & 1;
#pragma unroll
      for (int kwi = 0; kwi < KK; ++kwi) {
        const char* xs = px + ((vr0 + xr) * HWd + c * 16 + 8 * hfk + kwi + q) * PB + colb;
        const v4i16 x0 = ds_read_tr(xs);
        const v4i16 x1 = ds_read_tr(xs + 4 * PB);
        fb[kwi] = __builtin_bit_cast(uint4, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    };
    uint4 fbuf[2][KK];
    if constexpr (!(ABL & 2)) read_b(0, fbuf[0]);
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
      const int xr = st >> 1, c = st & 1;
      if constexpr (!(ABL & 2)) {
        if (st + 1 < NSTEP) read_b(st + 1, fbuf[(st + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const uint4* fb = fbuf[st & 1];
#pragma unroll
        for (int khi = KK - 1; khi >= 0; --khi) {
          const int r = xr - khi;
          if (r >= 0 && r < ROWS) {
#pragma unroll
            for (int kwi = 0; kwi < KK; ++kwi)
              if ((tmk >> (khi * KK + kwi)) & 1) mma<T>(acc[khi * KK + kwi], fa[r][c], fb[kwi]);
          }
        }
      }
      if constexpr (!(ABL & 1)) {
      // stage tile t+1 into the other buffer and refill its registers with
      // tile t+2: the dY chunks in the first step, the X chunks spread over
      // the rest (a past-the-end tile stages zeros nobody reads)
      if (st == 0) {
#pragma unroll
        for (int i = 0; i < MAXY; ++i) {
          commit_y(i, rg[i], nxt);
          rg[i] = load_chunk(i, rnn, have_nn);
        }
      }
#pragma unroll
      for (int j = 0; j < MAXX; ++j) {
        if ((j * NSTEP) / MAXX == st) {
          commit_x(j, rg[MAXY + j], nxt);
          rg[MAXY + j] = load_chunk(MAXY + j, rnn, have_nn);
        }
      }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    stage_i ^= 1;
    c0 = c1;
    c1 = c2;
    rn = rnn;
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
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int e = 0; e < 8; ++e) red[tid * 8 + e] = bsum[e];
    __syncthreads();
    if (tid < 32 * NCO) {
      // thread k's dY chunk position is k % YCPV: plane (k % YCPV) / 4, channels ((k % YCPV) % 4) * 8 + e
      const int plane = tid / 32, within = tid % 32;
      const int grp = plane * 4 + within / 8, e = within % 8;
      float sacc = 0.f;
      for (int kk = grp; kk < GTHR; kk += YCPV) sacc += red[kk * 8 + e];
      out[NW + tid] = sacc;
    }
  }
}

template <typename T, int NCO, int NCI, int PRO>
void launch_pipe(const WgradArgs& a, hipStream_t s) {
  const size_t lds = WpGeom<NCO, NCI>::lds_bytes();
  auto kern = conv_wgrad_pipe_kernel<T, NCO, NCI, PRO, 0>;
#ifdef VSRK_WP_EXP
  static int abl = -1;
  if (abl < 0) {
    const char* e = getenv("VSRK_WP_ABLATE");
    abl = e ? atoi(e) : 0;
  }
  if (abl == 1) kern = conv_wgrad_pipe_kernel<T, NCO, NCI, PRO, 1>;
  if (abl == 2) kern = conv_wgrad_pipe_kernel<T, NCO, NCI, PRO, 2>;
#endif
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<<<a.nblk, GTHR, lds, s>>>(a);
}

// prologue: none or BN-affine+ReLU (the DUF conv2 input); other modes take
// the generic kernel
template <typename T, int NCO, int NCI>
bool pipe_pro(const WgradArgs& a, hipStream_t s) {
  const int pro = a.prologue & (VSRK_PRO_AFFINE | VSRK_PRO_RELU);
  if (pro == 0) launch_pipe<T, NCO, NCI, 0>(a, s);
  else if (pro == (VSRK_PRO_AFFINE | VSRK_PRO_RELU)) launch_pipe<T, NCO, NCI, VSRK_PRO_AFFINE | VSRK_PRO_RELU>(a, s);
  else return false;
  return true;
}

template <typename T>
bool pipe_t(const WgradArgs& a, int nco, int nci, hipStream_t s) {
#ifdef VSRK_WP_EXP
  if (nco == 1 && nci == 2) return pipe_pro<T, 1, 2>(a, s);
  if (nco == 2 && nci == 2) return pipe_pro<T, 2, 2>(a, s);
  return false;
#else
  if (nco == 2 && nci == 2) return pipe_pro<T, 2, 2>(a, s);
  if (nco == 2) return pipe_pro<T, 2, 1>(a, s);
  if (nci == 2) return pipe_pro<T, 1, 2>(a, s);
  return pipe_pro<T, 1, 1>(a, s);
#endif
}

}  // namespace

int vsrk_g_wgrad_pipe_mode = -1;  // -1: from VSRK_WGRAD_PIPE (default on), 0 off, 1 on (vsrk_conv_set_path)

bool vsrk_wgrad_pipe_enabled() {
  int mode = vsrk_g_wgrad_pipe_mode;
  if (mode < 0) {
    const char* e = getenv("VSRK_WGRAD_PIPE");
    mode = (e && e[0] == '0') ? 0 : 1;
  }
  return mode != 0;
}

// 1 = launched (same slab layout as conv_wgrad_kernel); 0 = not eligible.
// Eligible: 16-bit, kh = kw = 3, chunk-readable views (plain or sub-pixel),
// whole 16-byte channel chunks, an (n, d) slice addressable in 30 bits.
int vsrk_conv_wgrad_pipe(const WgradArgs& a, int nco, int nci, int dtype, hipStream_t s) {
  if (!vsrk_wgrad_pipe_enabled()) return 0;
  if (a.kh != 3 || a.kw != 3) return 0;
  if (!a.xvec || !a.dyvec) return 0;
  if (a.cin % 8 || a.cout % 8 || a.x.cphys % 8 || a.dy.cphys % 8) return 0;
  const int64_t xs = ((int64_t)a.x.h * a.x.sh + (int64_t)a.x.w * a.x.sw) * 2 * a.x.r * a.x.r;
  const int64_t ys = ((int64_t)a.dy.h * a.dy.sh + (int64_t)a.dy.w * a.dy.sw) * 2 * a.dy.r * a.dy.r;
  if (xs >= (1ll << 30) || ys >= (1ll << 30)) return 0;
  if (a.x.sh < 0 || a.x.sw < 0 || a.dy.sh < 0 || a.dy.sw < 0) return 0;
  bool ok = false;
  if (dtype == VSRK_BF16) ok = pipe_t<bf16>(a, nco, nci, s);
#ifndef VSRK_WP_EXP
  else if (dtype == VSRK_F16) ok = pipe_t<f16>(a, nco, nci, s);
#endif
  return ok ? 1 : 0;
}

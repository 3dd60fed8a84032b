// Probe build of conv_k3 (VSRK_K3_DEBUG_DUMP): dump the first landed LDS
// stage of workgroup 0 and compare its B (weight) region with the packed
// weight it was loaded from.
#include <cstdio>
#include <vector>
__device__ char* g_dump;
#define VSRK_K3_DEBUG_DUMP g_dump
#define VSRK_K3_KERNEL_TU
#include "../../vsr_amd/csrc/conv_k3_impl.h"
using namespace vsrk_conv;
int vsrk_g_grid_cap = 0;
void vsrk_set_error(const char*, ...) {}
int vsrk_conv::k3_grid(int64_t n) { return (int)std::min<int64_t>(n, 512); }

int main() {
  const int N = 1, H = 16, W = 32, CI = 16, CO = 32, CIP = 32, COP = 128;
  std::vector<bf16> hx((size_t)N * H * W * CI), hw((size_t)9 * COP * CIP);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (bf16)(float)(i % 7);
  for (int tap = 0; tap < 9; ++tap)
    for (int co = 0; co < COP; ++co)
      for (int ci = 0; ci < CIP; ++ci) hw[((size_t)tap * COP + co) * CIP + ci] = (bf16)(float)(co < CO && ci < CI ? ((co * 7 + ci * 3) % 11) - 5 : 0);
  bf16 *dx, *dw, *dy;
  char* dd;
  hipMalloc(&dx, hx.size() * 2);
  hipMalloc(&dw, hw.size() * 2);
  hipMalloc(&dy, (size_t)N * H * W * CO * 2);
  hipMalloc(&dd, 1 << 20);
  hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dw, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  hipMemcpyToSymbol(HIP_SYMBOL(g_dump), &dd, sizeof(dd));
  vsrk_tensor5 xt{dx, N, 1, H, W, CI, (int64_t)H * W * CI, (int64_t)H * W * CI, W * CI, CI, 1, VSRK_BF16};
  vsrk_tensor5 yt{dy, N, 1, H, W, CO, (int64_t)H * W * CO, (int64_t)H * W * CO, W * CO, CO, 1, VSRK_BF16};
  K3Args a{};
  a.x = make_view(&xt); a.y = make_view(&yt); a.res = a.y; a.msk = a.y;
  a.w = dw; a.cin = CI; a.cout = CO; a.cin_pad = CIP; a.cout_pad = COP;
  a.kd = 1; a.pd = 0; a.ph = 1; a.pw = 1; a.out_scale = 1.f;
  a.tiles_w = 1; a.ntn = 1;
  int rc = launch_k3<32, 0, 0, 0>(a, 0);
  hipError_t e = hipDeviceSynchronize();
  printf("rc %d status %s\n", rc, hipGetErrorString(e));
  using G = K3Geom<32>;
  std::vector<bf16> dump(G::SLOT / 2);
  hipMemcpy(dump.data(), dd, G::SLOT, hipMemcpyDeviceToHost);
  const bf16* B = dump.data() + K3_ABYTES / 2;
  int bad = 0;
  for (int pl = 0; pl < 2; ++pl)
    for (int tap = 0; tap < 9; ++tap)
      for (int co = 0; co < 32; ++co) {
        const bf16* ent = B + ((size_t)pl * G::BENT + tap * 32 + co) * 8;
        for (int e = 0; e < 8; ++e) {
          float want = (float)(((co * 7 + (8 * pl + e) * 3) % 11) - 5), got = (float)ent[e];
          if (got != want && bad++ < 12) printf("B pl %d tap %d co %d e %d: got %g want %g\n", pl, tap, co, e, got, want);
        }
      }
  printf("B region mismatches: %d of %d\n", bad, 2 * 9 * 32 * 8);
  const bf16* A = dump.data();
  int abad = 0;
  for (int pl = 0; pl < 2; ++pl)
    for (int hh = 0; hh < 18; ++hh)
      for (int ww = 0; ww < 34; ++ww) {
        const bf16* ent = A + ((size_t)pl * K3_NVP + hh * 34 + ww) * 8;
        const int h = hh - 1, w = ww - 1;
        for (int e = 0; e < 8; ++e) {
          float want = (h < 0 || h >= H || w < 0 || w >= W) ? 0.f : (float)hx[((size_t)h * W + w) * CI + 8 * pl + e];
          if ((float)ent[e] != want && abad++ < 6) printf("A pl %d (%d,%d) e %d: got %g want %g\n", pl, hh, ww, e, (float)ent[e], want);
        }
      }
  printf("A region mismatches: %d\n", abad);
  // output at voxel (5, 7) vs a host conv (identity-free check of the MFMA + epilogue)
  std::vector<bf16> hy((size_t)N * H * W * CO);
  hipMemcpy(hy.data(), dy, hy.size() * 2, hipMemcpyDeviceToHost);
  for (int vh : {5}) for (int vw : {0, 7, 31}) {
    printf("y(%d,%d):", vh, vw);
    for (int c = 0; c < 32; ++c) printf(" %g", (float)hy[((size_t)vh * W + vw) * CO + c]);
    printf("\nref  :");
    for (int c = 0; c < 32; ++c) {
      double s = 0;
      for (int kh = 0; kh < 3; ++kh) for (int kw = 0; kw < 3; ++kw) {
        const int h = vh + kh - 1, w = vw + kw - 1;
        if (h < 0 || h >= H || w < 0 || w >= W) continue;
        for (int ci = 0; ci < CI; ++ci)
          s += (double)(float)hx[((size_t)h * W + w) * CI + ci] * (double)(float)hw[((size_t)(kh * 3 + kw) * COP + c) * CIP + ci];
      }
      printf(" %g", s);
    }
    printf("\n");
  }
  return 0;
}

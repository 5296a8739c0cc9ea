// The 2x2 stride-2 convolutions as streaming GEMMs with the weights resident in
// registers (gfx950, round 6): written for DownsampleBlock's conv (Unet_model.py:26-30),
// UpsampleBlock's transposed conv (:36-42) and their input gradients (the transposed
// conv's is a 2x2 / s2 gather, the down conv's a per-pixel GEMM scattered to 2x2), bf16;
// it runs where it measured faster (rdn_conv_pix_launch: the level-0 down conv's input
// gradient).  K = taps * cin is small (64-256) and every output pixel is written once,
// so these launches are HBM-bound: conv_gemm.hip's tiles (K through a double-buffered
// LDS stage, the fp32 tile staged through LDS for the epilogue, 80 KB per block, two
// blocks per CU) ran them at 1.4-3.9 TB/s.  Here there is no LDS and no barrier:
//
// * a wave owns 16 * CT output columns and keeps their weights (the MFMA A operand,
//   CT x KS fragments of 16 columns x 32 k, 4 VGPRs each) in registers for the launch;
// * it streams pairs of 16-pixel groups: the B operand (32 k x 16 pixels) is gathered
//   straight from the NHWC / channel-blocked input into registers (16 B per lane: 8
//   consecutive k of one tap of one pixel), v_mfma_f32_16x16x32_bf16 leaves a lane 4
//   channels of one pixel, and v_permlane16_swap between the two groups' accumulators
//   gives it 8 consecutive channels -- one 16-byte unit per store, with bias, PReLU
//   input, PReLU, residual / accumulate and the depth-to-space scatter applied in
//   registers;
// * waves are persistent (a grid of ~8 per SIMD); the waves of one 16-pixel stream but
//   different column slices are consecutive logical blocks, placed on one XCD
//   (xcd_remap), so the repeated input reads hit its L2.
//
// Same operands, same k order and the same MFMA as conv_gemm_kernel with the operands
// swapped (D = W x^T instead of x W^T): every output element is the same 32-term
// dot products accumulated in the same k-step order (bit-identical results,
// tests/test_gpu_pix.py).
#include "rdn_common.h"

namespace {

constexpr int NT = 256;

template <int CT, int KS, int GATHER>
__global__ __launch_bounds__(NT) void conv_pix_kernel(rdn_conv_desc d, int ncs, int streams, int groups, FastDiv fd_w,
                                                      FastDiv fd_hw) {
  const int lane = threadIdx.x & 63;
  const int gw = xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
  const int cs = gw % ncs, s = gw / ncs;
  if (s >= streams) return;   // whole waves; no barrier in this kernel
  const int r = lane & 15, g = lane >> 4;
  const int n0 = cs * (16 * CT);
  const int64_t M = (int64_t)d.n * d.h * d.w;
  const bf16* __restrict__ X = (const bf16*)d.x;

  // ---- weights of this wave's columns, all of K: A[col n0 + 16 ct + r][k = 32 ks + 8 g ..]
  u32x4 wa[CT][KS];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wa[ct][ks] = *(const u32x4*)((const bf16*)d.wp + (int64_t)(n0 + 16 * ct + r) * d.kp + 32 * ks + 8 * g);

  // ---- this lane's k units: tap and channel offset per k-step (k = tap * cin + ci)
  int ktap[KS];
  int64_t kcf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k = 32 * ks + 8 * g;
    const int tap = GATHER == RDN_G_S2 ? k / d.cin : 0, ci = k - tap * d.cin;
    ktap[ks] = tap;
    kcf[ks] = rdn_coff(d.x_c0 + ci, d.x_ps, d.x_pl);
  }

  // the B fragments of a 16-pixel group: pixel m0 + r, 8 k of each k-step
  auto gather = [&](int64_t m, u32x4 (&bx)[KS]) {
    const bool ok = m < M;
    const uint32_t mm = ok ? (uint32_t)m : 0u;
    int64_t pb;   // source pixel of tap 0
    if constexpr (GATHER == RDN_G_S2) {
      const uint32_t nimg = fdiv(mm, fd_hw), rem = mm - nimg * (uint32_t)(d.h * d.w);
      const uint32_t y = fdiv(rem, fd_w), x = rem - y * (uint32_t)d.w;
      pb = ((int64_t)nimg * d.hin + 2 * y) * d.win + 2 * x;
    } else {
      pb = mm;
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int64_t px = GATHER == RDN_G_S2 ? pb + (int64_t)(ktap[ks] >> 1) * d.win + (ktap[ks] & 1) : pb;
      bx[ks] = ok ? *(const u32x4*)(X + px * d.x_ps + kcf[ks]) : u32x4{0u, 0u, 0u, 0u};
    }
  };

  const int flags = d.flags;
  const int H = d.h, W = d.w;
  u32x4 bx[2][KS];
  int it = s;
  if (it < groups) {
    gather((int64_t)it * 32 + r, bx[0]);
    gather((int64_t)it * 32 + 16 + r, bx[1]);
  }
  for (; it < groups; it += streams) {
    f32x4 acc[2][CT];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wa[ct][ks]),
                                                      __builtin_bit_cast(bf16x8, bx[h][ks]), a, 0, 0, 0);
        acc[h][ct] = a;
      }
    // the next pair's gathers are in flight during this pair's epilogue
    const int nit = it + streams;
    if (nit < groups) {
      gather((int64_t)nit * 32 + r, bx[0]);
      gather((int64_t)nit * 32 + 16 + r, bx[1]);
    }
    // lane (r, g): channels 16 ct + 8 (g >> 1) .. + 7 of pixel it * 32 + 16 (g & 1) + r
    // (every lane takes part in the swaps below; a lane past the last pixel stores nothing)
    const int64_t m = (int64_t)it * 32 + 16 * (g & 1) + r;
    const bool mok = m < M;
    int64_t opix = m;
    int tapo = 0;
    int oy = 0, ox = 0, onimg = 0;
    if (flags & RDN_EPI_SCATTER2) {
      const uint32_t mm = mok ? (uint32_t)m : 0u;
      const uint32_t nimg = fdiv(mm, fd_hw), rem = mm - nimg * (uint32_t)(H * W);
      const uint32_t y = fdiv(rem, fd_w), x = rem - y * (uint32_t)W;
      onimg = (int)nimg; oy = (int)y; ox = (int)x;
    }
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const u32x4 ua = __builtin_bit_cast(u32x4, acc[0][ct]), ub = __builtin_bit_cast(u32x4, acc[1][ct]);
      u32x4 lo, hi;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto sw = __builtin_amdgcn_permlane16_swap(ua[e], ub[e], false, false);
        lo[e] = sw[0];
        hi[e] = sw[1];
      }
      const f32x4 flo = __builtin_bit_cast(f32x4, lo), fhi = __builtin_bit_cast(f32x4, hi);
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = flo[e];
        v[4 + e] = fhi[e];
      }
      if (!mok) continue;
      const int col = n0 + 16 * ct + 8 * (g >> 1);
      int c = col;
      if (flags & RDN_EPI_SCATTER2) {   // column tap * cout + c -> pixel (2y + dy, 2x + dx)
        tapo = col / d.cout;
        c = col - tapo * d.cout;
        opix = ((int64_t)onimg * (2 * H) + 2 * oy + (tapo >> 1)) * (2 * W) + 2 * ox + (tapo & 1);
      }
      if (flags & RDN_EPI_BIAS) {
        const f32x4 b0 = *(const f32x4*)(d.bias + c), b1 = *(const f32x4*)(d.bias + c + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] += b0[e];
          v[4 + e] += b1[e];
        }
      }
      if (flags & RDN_EPI_STORE_PRE)
        *(u32x4*)((bf16*)d.pre + opix * d.pre_ps + rdn_coff(c, d.pre_ps, d.pre_pl)) = Unit16<bf16>::pack(v);
      if (flags & RDN_EPI_PRELU) {
        const f32x4 a0 = *(const f32x4*)(d.alpha + c), a1 = *(const f32x4*)(d.alpha + c + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = v[e] > 0.f ? v[e] : a0[e] * v[e];
          v[4 + e] = v[4 + e] > 0.f ? v[4 + e] : a1[e] * v[4 + e];
        }
      }
      bf16* const op = (bf16*)d.out + opix * d.out_ps + rdn_coff(d.out_c0 + c, d.out_ps, d.out_pl);
      float rv[8];
      if ((flags & RDN_EPI_RESID) && c < d.res_climit) {
        Unit16<bf16>::unpack(*(const u32x4*)((const bf16*)d.res + opix * d.res_ps +
                                             rdn_coff(d.res_c0 + c, d.res_ps, d.res_pl)), rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += rv[e];
      }
      if (flags & RDN_EPI_ACCUM) {
        Unit16<bf16>::unpack(*(const u32x4*)op, rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += rv[e];
      }
      *(u32x4*)op = Unit16<bf16>::pack(v);
    }
  }
}

template <int CT, int KS>
int launch_pix(const rdn_conv_desc* d, hipStream_t st) {
  const int64_t M = (int64_t)d->n * d->h * d->w;
  const int ncs = d->ncols / (16 * CT);
  const int64_t groups = (M + 31) / 32;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  // persistent: as many waves as are resident (a stream = ncs waves)
  static int bpc[2] = {0, 0};
  int& res = bpc[d->gather == RDN_G_S2];
  if (!res) {
    int n = 0;
    if (d->gather == RDN_G_S2)
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv_pix_kernel<CT, KS, RDN_G_S2>, NT, 0);
    else
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv_pix_kernel<CT, KS, RDN_G_PIX>, NT, 0);
    res = n > 0 ? n : 1;
  }
  int64_t streams = (int64_t)cus * res * 4 / ncs;
  if (streams > groups) streams = groups;
  if (streams < 1) streams = 1;
  const int64_t blocks = (streams * ncs + 3) / 4;
  FastDiv fw = make_fastdiv((uint32_t)d->w), fhw = make_fastdiv((uint32_t)(d->h * d->w));
  RDN_PROBE("conv_pix_kernel<bf16,%d,%d,%d>", CT, KS, d->gather);
  if (d->gather == RDN_G_S2)
    conv_pix_kernel<CT, KS, RDN_G_S2><<<(unsigned)blocks, NT, 0, st>>>(*d, ncs, (int)streams, (int)groups, fw, fhw);
  else
    conv_pix_kernel<CT, KS, RDN_G_PIX><<<(unsigned)blocks, NT, 0, st>>>(*d, ncs, (int)streams, (int)groups, fw, fhw);
  return rdn_check_launch("rdn_conv_fwd(conv pix)");
}

}  // namespace

// The 2x2 / s2 and per-pixel GEMMs of bf16 launches with K = taps * cin in {64, 128,
// 256} and 64-column multiples, 16-byte units everywhere; 1 = not this kernel's shape
// (conv_gemm.hip then runs it).
int rdn_conv_pix_launch(const rdn_conv_desc* d, hipStream_t st) {
  if (d->dtype != RDN_BF16 || (d->gather != RDN_G_S2 && d->gather != RDN_G_PIX) || d->gate || d->gout) return 1;
  if (d->flags & ~(RDN_EPI_BIAS | RDN_EPI_STORE_PRE | RDN_EPI_PRELU | RDN_EPI_RESID | RDN_EPI_ACCUM | RDN_EPI_SCATTER2))
    return 1;
  if (d->bm || d->bn) return 1;
  const int taps = d->gather == RDN_G_S2 ? 4 : 1;
  const int K = taps * d->cin;
  if (d->cin % 8 || d->ncols % 64 || d->x_ps % 8 || d->x_c0 % 8 || d->out_ps % 8 || d->out_c0 % 8 || d->kp < K ||
      ((uintptr_t)d->x & 15) || ((uintptr_t)d->wp & 15) || ((uintptr_t)d->out & 15))
    return 1;
  if ((d->flags & RDN_EPI_STORE_PRE) && (d->pre_ps % 8 || ((uintptr_t)d->pre & 15))) return 1;
  if ((d->flags & RDN_EPI_RESID) && (d->res_ps % 8 || d->res_c0 % 8 || d->res_climit % 8 || ((uintptr_t)d->res & 15)))
    return 1;
  if ((d->flags & RDN_EPI_SCATTER2) && (d->cout % 16 || d->cout * 4 != d->ncols)) return 1;
  if ((int64_t)d->n * d->h * d->w >= (1ll << 31)) return 1;
  // Where it runs (per-layer A/B against conv_gemm_kernel in the B16 train step, r06,
  // bit-identical either way): the K = 64 per-pixel GEMM without a PReLU-input store --
  // the down_0 input gradient, 58.6 -> 42.8 us.  Measured and left on conv_gemm: the
  // K = 64 transposed-conv forward with its PReLU-input stores (up_0.conv_t 76.7 -> 83.1
  // us), the K = 128 shapes (CT = 2: down_0 40.7 -> 39.0, up_1.conv_t 60.2 -> 61.7, down_1
  // dgrad 36.8 -> 37.8) and the K = 256 ones (CT = 1, 16-column waves re-reading every
  // pixel 16-32 times: up_2.conv_t 36.9 -> 77.6, down_2 dgrad 22.6 -> 44.6 us).
  if (K == 64 && d->gather == RDN_G_PIX && !(d->flags & RDN_EPI_STORE_PRE)) return launch_pix<4, 2>(d, st);
  return 1;
}

// Image-quality metrics of the SIDD evaluation, batched on
// the GPU.  The reference evaluates per image on the host with scikit-image
// 0.22 (requirements.txt:98):
//
//   peak_signal_noise_ratio(gt, out, data_range=2)                 evaluate_SIDD/evaluate_SIDD.py:63
//   structural_similarity(gt, out, data_range=2, channel_axis=-1)  evaluate_SIDD/evaluate_SIDD.py:64
//
// after moving every denoised block to the host (.cpu().numpy(), :59-61).  Here
// both metrics of a whole batch come out of one pass over the two fp32 NCHW
// images in HBM.
//
// skimage semantics restated (oracle/metrics_ref.py has the numpy form):
//   PSNR = 10 log10(R^2 / mse), mse = mean((gt - x)^2) over C*H*W (fp32
//          difference, float64 sum), inf when mse == 0.
//   SSIM per channel: 7x7 uniform means (scipy uniform_filter) of x, y, x^2, y^2,
//          xy; vx = cov_norm (uxx - ux^2), cov_norm = 49/48 (sample covariance);
//          C1 = (0.01 R)^2, C2 = (0.03 R)^2;
//          S = (2 ux uy + C1)(2 vxy + C2) / ((ux^2 + uy^2 + C1)(vx + vy + C2));
//          mean of S over the interior (3 pixels cropped on every side, where the
//          7x7 window never leaves the image, so the filter's border mode never
//          enters the result); the image SSIM is the mean over channels.
//
// Block = up to 506 output columns x 16-64 rows of one (image, channel) plane,
// streamed row by row (see the kernel).  Per-block (squared error, sum S) partials in
// float64; a second launch sums them per image in a fixed order (deterministic).
// HBM-bound: 8 bytes per pixel read once (+6 columns, +6 rows of halo per tile).
#include "rdn_common.h"

#include <math.h>

namespace {

constexpr int NT_MAX = 512;
constexpr int R = 3, WIN = 2 * R + 1;
constexpr int TY_MAX = 64;        // output rows per block

// column tiling: tiles of txo output columns, blockDim = roundup(txo + 6, 64) <= 512
// threads (one input column each): a 256-wide SIDD block is ONE tile of 320 threads
struct ColTiles { int n, txo, nt; };
ColTiles col_tiles(int w) {
  ColTiles c;
  c.n = (w + (NT_MAX - 2 * R) - 1) / (NT_MAX - 2 * R);
  c.txo = (w + c.n - 1) / c.n;
  c.nt = (c.txo + 2 * R + 63) / 64 * 64;
  return c;
}

// Block = txo output columns x TY output rows of one (image, channel) plane; thread
// t owns input column ox0 - 3 + t.  The block walks its TY + 6 input rows once: each
// row goes to a double-buffered LDS row of (gt, x) pairs (one barrier per row), thread
// t < txo forms the horizontal 7-sums of the five moments (u, v, u^2, v^2, uv) of output
// column ox0 + t, keeps the last 7 rows of them in registers and a running window sum
// (add the new row, subtract the one it replaces: 6 VALU per row instead of the 21 of a
// fresh 7-row sum; fp32 over <= 70 rows, scipy's uniform_filter also slides a running
// sum); the next 7 rows' loads are in flight meanwhile.
// The kernel is VALU-issue bound, so the moments go as packed fp32
// pairs -- (u, v) and (u^2, v^2) by one v_pk_add_f32 / v_pk_fma_f32 each, in the same
// per-lane order and rounding as the scalar form -- the SSIM quotient takes one
// reciprocal (1 ulp) instead of the IEEE division sequence, and a thread's squared
// errors and SSIM terms (<= 64 rows) are summed in fp32 and widened to float64 once,
// for the block's float64 reduction.  Held to 5 waves per SIMD (94 VGPRs; the
// unconstrained build took 164 and ran 3 per SIMD, too few to keep the row loads in
// flight).  64 x 3 x 256^2 block pairs: 79 -> 48.5 us, 0.16 -> 0.26 of HBM (r06,
// PMC: VALU instructions -34 %, wave cycles -31 %).
__global__ __launch_bounds__(NT_MAX, 5) void image_metrics_kernel(const float* __restrict__ gt,
                                                               const float* __restrict__ x, int C, int H, int W,
                                                               int tiles_x, int TXO, int TY, float c1, float c2,
                                                               float cov_norm, double* __restrict__ part) {
  __shared__ f32x2 rowbuf[2][NT_MAX];
  __shared__ double red[2][NT_MAX / 64];
  const int t = threadIdx.x;
  const int tile = blockIdx.x, c = blockIdx.y, n = blockIdx.z;
  const int ox0 = (tile % tiles_x) * TXO, oy0 = (tile / tiles_x) * TY;
  const int64_t plane = ((int64_t)n * C + c) * H * W;
  const float* __restrict__ ga = gt + plane;
  const float* __restrict__ gb = x + plane;
  const int xi = ox0 - R + t;                       // this thread's input column
  const bool xin = (unsigned)xi < (unsigned)W;
  const bool own_x = t >= R && t < R + TXO && xi < W;          // PSNR: pixels of this tile only
  const int xo = ox0 + t;                                      // output column of thread t < TXO
  const bool ssim_x = t < TXO && xo >= R && xo < W - R;
  const int rows = TY + 2 * R;
  const int y_lo = oy0 > R ? oy0 : R, y_hi = (oy0 + TY < H - R) ? oy0 + TY : H - R;   // SSIM rows

  // buffer loads: a pixel outside the image (or past the last row) reads at an offset
  // past the descriptor's range, which returns 0 -- no select after the load, so each
  // row's value is waited for only where it is consumed and the 7-row prefetch stays
  // in flight (a clamped load + select made hipcc wait for all seven at once)
  const __amdgpu_buffer_rsrc_t rsa = rdn_rsrc(ga), rsb = rdn_rsrc(gb);
  auto load = [&](int r, float& a, float& b) {
    const int y = oy0 - R + r;
    const bool in = xin && (unsigned)y < (unsigned)H && r < rows;
    int o = in ? (y * W + xi) * 4 : RDN_OOB;
    asm volatile("" : "+v"(o));
    a = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsa, o, 0, 0));
    b = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsb, o, 0, 0));
  };
  // rows r .. r+6 in flight: slot k of the register ring holds row r0 + k
  f32x2 h01[WIN], h23[WIN];
  float h4[WIN];
#pragma unroll
  for (int k = 0; k < WIN; ++k) {
    h01[k] = f32x2{0.f, 0.f};
    h23[k] = f32x2{0.f, 0.f};
    h4[k] = 0.f;
  }
  float se = 0.f, ss = 0.f;
  f32x2 m01 = {0.f, 0.f}, m23 = {0.f, 0.f};   // window sums of the last 7 rows' horizontal sums
  float m4 = 0.f;
  float pa[WIN], pb[WIN];
#pragma unroll
  for (int k = 0; k < WIN; ++k) load(k, pa[k], pb[k]);
  const f32x2 inv2 = {1.f / (WIN * WIN), 1.f / (WIN * WIN)};
  for (int r0 = 0; r0 < rows; r0 += WIN) {
#pragma unroll
    for (int k = 0; k < WIN; ++k) {
      const int r = r0 + k;
      if (r < rows) {   // uniform across the block
        const float a = pa[k], b = pb[k];
        load(r + WIN, pa[k], pb[k]);
        const int y = oy0 - R + r;
        if (own_x && y >= oy0 && y < oy0 + TY && y < H) {
          const float d = a - b;
          se += d * d;
        }
        f32x2* const rb = rowbuf[r & 1];
        rb[t] = f32x2{a, b};
        __syncthreads();
        if (t < TXO) {
          f32x2 s01 = {0.f, 0.f}, s23 = {0.f, 0.f};
          float s4 = 0.f;
#pragma unroll
          for (int q = 0; q < WIN; ++q) {
            const f32x2 uv = rb[t + q];
            s01 += uv;
            s23 += uv * uv;
            s4 = __builtin_fmaf(uv[0], uv[1], s4);
          }
          // running 7-row window sums: add row r, drop row r - 7 (the ring slot it replaces)
          m01 += s01 - h01[k];
          m23 += s23 - h23[k];
          m4 += s4 - h4[k];
          h01[k] = s01; h23[k] = s23; h4[k] = s4;
          const int yo = y - R;                 // output row whose window just completed
          if (r >= 2 * R && ssim_x && yo >= y_lo && yo < y_hi) {
            const f32x2 u = m01 * inv2;                       // (ux, uy)
            const f32x2 v = cov_norm * (m23 * inv2 - u * u);  // (vx, vy)
            const float vxy = cov_norm * (m4 * inv2[0] - u[0] * u[1]);
            const float a1 = 2.f * u[0] * u[1] + c1, a2 = 2.f * vxy + c2;
            const float b1 = u[0] * u[0] + u[1] * u[1] + c1, b2 = v[0] + v[1] + c2;
            ss += (a1 * a2) * __builtin_amdgcn_rcpf(b1 * b2);
          }
        }
      }
    }
  }
  // block reduction in float64 (wave shuffles, then the wave sums in a fixed order)
  double sed = (double)se, ssd = (double)ss;
  for (int o = 32; o > 0; o >>= 1) {
    sed += __shfl_down(sed, o, 64);
    ssd += __shfl_down(ssd, o, 64);
  }
  if ((t & 63) == 0) { red[0][t >> 6] = sed; red[1][t >> 6] = ssd; }
  __syncthreads();
  if (t == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < (int)(blockDim.x / 64); ++w) { a += red[0][w]; b += red[1][w]; }
    const int64_t slot = ((int64_t)n * C + c) * gridDim.x + tile;
    part[2 * slot] = a;
    part[2 * slot + 1] = b;
  }
}

// one block per image: thread t sums slots t, t + 256, ... of the image's C x tiles
// partials, then a fixed shared-memory tree (deterministic).  (One thread per image
// looping over its slots waits on C x tiles dependent loads.)
__global__ __launch_bounds__(256) void image_metrics_final_kernel(const double* __restrict__ part, int C, int H,
                                                                  int W, int tiles, double range,
                                                                  double* __restrict__ psnr, double* __restrict__ ssim) {
  __shared__ double red[2][256];
  const int n = blockIdx.x, t = threadIdx.x;
  const int slots = C * tiles;
  double se = 0.0, sc = 0.0;
  for (int k = t; k < slots; k += 256) {
    const int64_t slot = (int64_t)n * slots + k;
    se += part[2 * slot];
    sc += part[2 * slot + 1];
  }
  red[0][t] = se;
  red[1][t] = sc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      red[0][t] += red[0][t + o];
      red[1][t] += red[1][t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    const double interior = (double)(H - 2 * R) * (double)(W - 2 * R);
    const double mse = red[0][0] / ((double)C * H * W);
    if (psnr) psnr[n] = 10.0 * log10(range * range / mse);   // mse == 0 -> inf, as skimage
    if (ssim) ssim[n] = red[1][0] / interior / C;
  }
}

// rows per block: fewer, taller tiles measured faster than a fuller grid of short
// ones (the 6 halo rows are re-read per tile): 64 rows -> 75 us, 16 rows -> 113 us
// for 64 x 3 x 256^2 block pairs on MI355X
int row_tile(int, int, int, int) { return TY_MAX; }

int tiles_of(int n, int c, int h, int w) {
  const int ty = row_tile(n, c, h, w);
  return col_tiles(w).n * ((h + ty - 1) / ty);
}

}  // namespace

extern "C" int64_t rdn_image_metrics_workspace_size(int32_t n, int32_t c, int32_t h, int32_t w) {
  if (n <= 0 || c <= 0 || h <= 0 || w <= 0) return 0;
  return (int64_t)n * c * tiles_of(n, c, h, w) * 2 * (int64_t)sizeof(double);
}

extern "C" int rdn_image_metrics(const float* gt, const float* x, int32_t n, int32_t c, int32_t h, int32_t w,
                                 float data_range, double* ws, double* psnr, double* ssim, void* stream) {
  if (!gt || !x || !ws || (!psnr && !ssim)) { rdn_set_error("rdn_image_metrics: null pointer"); return RDN_E_ARG; }
  if (n <= 0 || c <= 0 || n > 65535 || c > 65535) { rdn_set_error("rdn_image_metrics: bad n=%d c=%d", n, c); return RDN_E_SHAPE; }
  if (h < WIN || w < WIN) {   // skimage: win_size exceeds image extent
    rdn_set_error("rdn_image_metrics: images must be at least %dx%d (got %dx%d)", WIN, WIN, h, w);
    return RDN_E_SHAPE;
  }
  if (!(data_range > 0.f)) { rdn_set_error("rdn_image_metrics: data_range must be > 0"); return RDN_E_ARG; }
  if ((int64_t)h * w >= (1ll << 29)) { rdn_set_error("rdn_image_metrics: planes of 2^29 pixels or more"); return RDN_E_SHAPE; }
  const ColTiles ct = col_tiles(w);
  const int tiles = tiles_of(n, c, h, w), ty = row_tile(n, c, h, w);
  const double rr = data_range;
  const float c1 = (float)((0.01 * rr) * (0.01 * rr)), c2 = (float)((0.03 * rr) * (0.03 * rr));
  const float cov_norm = (float)(WIN * WIN) / (float)(WIN * WIN - 1);
  image_metrics_kernel<<<dim3(tiles, c, n), ct.nt, 0, (hipStream_t)stream>>>(gt, x, c, h, w, ct.n, ct.txo, ty, c1, c2,
                                                                             cov_norm, ws);
  image_metrics_final_kernel<<<n, 256, 0, (hipStream_t)stream>>>(ws, c, h, w, tiles, rr, psnr, ssim);
  return rdn_check_launch("rdn_image_metrics");
}

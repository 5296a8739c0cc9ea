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
// row goes to a double-buffered LDS row (one barrier per row), thread t < txo
// forms the horizontal 7-sums of the five moments (u, v, u^2, v^2, uv) of output
// column ox0 + t, keeps the last 7 rows of them in registers and sums those
// (no running-sum subtraction: each window mean is a fresh 49-term sum, as
// exact as the oracle's); the next 7 rows' loads are in flight meanwhile.
__global__ __launch_bounds__(NT_MAX) void image_metrics_kernel(const float* __restrict__ gt,
                                                               const float* __restrict__ x, int C, int H, int W,
                                                               int tiles_x, int TXO, int TY, float c1, float c2,
                                                               float cov_norm, double* __restrict__ part) {
  __shared__ float rowbuf[2][2][NT_MAX];
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

  // unconditional loads from a clamped (always valid) address, zeroed after:
  // a load under a branch makes hipcc wait vmcnt(0) for it, which would drain
  // the 7-row prefetch every row
  const int xc = xi < 0 ? 0 : (xi >= W ? W - 1 : xi);
  auto load = [&](int r, float& a, float& b) {
    const int y = oy0 - R + r;
    const bool in = xin && (unsigned)y < (unsigned)H && r < rows;
    const int yc = y < 0 ? 0 : (y >= H ? H - 1 : y);
    const float va = ga[(int64_t)yc * W + xc], vb = gb[(int64_t)yc * W + xc];
    a = in ? va : 0.f;
    b = in ? vb : 0.f;
  };
  // rows r .. r+6 in flight: slot k of the register ring holds row r0 + k
  float h[WIN][5];
#pragma unroll
  for (int k = 0; k < WIN; ++k)
#pragma unroll
    for (int j = 0; j < 5; ++j) h[k][j] = 0.f;
  double se = 0.0, ss = 0.0;
  float pa[WIN], pb[WIN];
#pragma unroll
  for (int k = 0; k < WIN; ++k) load(k, pa[k], pb[k]);
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
          se += (double)(d * d);
        }
        float* const ra = rowbuf[r & 1][0];
        float* const rb = rowbuf[r & 1][1];
        ra[t] = a;
        rb[t] = b;
        __syncthreads();
        if (t < TXO) {
          float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
#pragma unroll
          for (int q = 0; q < WIN; ++q) {
            const float u = ra[t + q], v = rb[t + q];
            s0 += u; s1 += v; s2 += u * u; s3 += v * v; s4 += u * v;
          }
          h[k][0] = s0; h[k][1] = s1; h[k][2] = s2; h[k][3] = s3; h[k][4] = s4;
          const int yo = y - R;                 // output row whose window just completed
          if (r >= 2 * R && ssim_x && yo >= y_lo && yo < y_hi) {
            float m[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
              float acc = 0.f;
#pragma unroll
              for (int q = 0; q < WIN; ++q) acc += h[(k + 1 + q) % WIN][j];   // rows yo-3 .. yo+3 in order
              m[j] = acc;
            }
            constexpr float inv = 1.f / (WIN * WIN);
            const float ux = m[0] * inv, uy = m[1] * inv;
            const float vx = cov_norm * (m[2] * inv - ux * ux);
            const float vy = cov_norm * (m[3] * inv - uy * uy);
            const float vxy = cov_norm * (m[4] * inv - ux * uy);
            const float a1 = 2.f * ux * uy + c1, a2 = 2.f * vxy + c2;
            const float b1 = ux * ux + uy * uy + c1, b2 = vx + vy + c2;
            ss += (double)((a1 * a2) / (b1 * b2));
          }
        }
      }
    }
  }
  // block reduction (wave shuffles, then the 4 wave sums in a fixed order)
  for (int o = 32; o > 0; o >>= 1) {
    se += __shfl_down(se, o, 64);
    ss += __shfl_down(ss, o, 64);
  }
  if ((t & 63) == 0) { red[0][t >> 6] = se; red[1][t >> 6] = ss; }
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

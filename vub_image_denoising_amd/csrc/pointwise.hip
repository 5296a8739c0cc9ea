// Memory-bound kernels of the diffusion-RDUNet train/sample step (gfx950).
// Each is a single pass over HBM with 16-byte accesses where the layout
// allows; reductions go wave shuffle -> LDS -> one atomic (or one partial)
// per block.
#include <stdarg.h>
#include <stdio.h>

#include "rdn_common.h"

// ------------------------------------------------------------------ errors
static thread_local char g_err[512] = "";
void rdn_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
int rdn_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    rdn_set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return RDN_E_LAUNCH;
  }
  return RDN_OK;
}
extern "C" const char* rdn_last_error(void) { return g_err; }

thread_local char* rdn_probe_buf = nullptr;
thread_local int rdn_probe_len = 0;
thread_local int rdn_probe_rows = 0;
int rdn_probe_name(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(rdn_probe_buf, (size_t)rdn_probe_len, fmt, ap);
  va_end(ap);
  return RDN_OK;
}
extern "C" int rdn_conv_kernel_name(const rdn_conv_desc* d, char* buf, int32_t len) {
  if (!buf || len < 1) { rdn_set_error("rdn_conv_kernel_name: no buffer"); return RDN_E_ARG; }
  buf[0] = 0;
  rdn_probe_buf = buf;
  rdn_probe_len = len;
  const int rc = rdn_conv_fwd(d, nullptr);
  rdn_probe_buf = nullptr;
  return rc;
}
extern "C" int rdn_conv_gate_rows(const rdn_conv_desc* d) {
  if (!d || !d->gout) return 0;
  char buf[128];
  rdn_probe_buf = buf;
  rdn_probe_len = (int)sizeof(buf);
  rdn_probe_rows = 0;
  const int rc = rdn_conv_fwd(d, nullptr);
  rdn_probe_buf = nullptr;
  return rc == RDN_OK ? rdn_probe_rows : 0;
}
extern "C" int rdn_wgrad_kernel_name(const rdn_wgrad_desc* d, char* buf, int32_t len) {
  if (!buf || len < 1) { rdn_set_error("rdn_wgrad_kernel_name: no buffer"); return RDN_E_ARG; }
  buf[0] = 0;
  rdn_probe_buf = buf;
  rdn_probe_len = len;
  const int rc = rdn_conv_wgrad(d, nullptr);
  rdn_probe_buf = nullptr;
  return rc;
}
extern "C" const char* rdn_version(void) { return "rdunet_hip 0.1.0 gfx950"; }

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int RDN_PRELU_PU = 4;   // pixel iterations per trip of the NHWC fast path

static int grid_for(int64_t n, int per_block, int cap = 8192) {
  int64_t b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

// ------------------------------------------------------------------ PReLU bwd
// dyp = dy * (pre > 0 ? 1 : a);  dalpha += sum_{pre<=0} pre*dy;  dbias += sum dyp
// (aten prelu backward: mask = input > 0, Activation.cpp; conv grad_bias = sum
// over N,H,W of grad_output).  Thread = 16-byte channel group of one pixel.
template <typename T>
// (<= 64 VGPRs: one wave per SIMD still fits beside a two-wave weight-gradient block of
// the side stream -- 2 x 218 of 512 -- so the pass is not confined to the CUs the
// side stream leaves free)
__global__ __launch_bounds__(256, 1) void prelu_bwd_kernel(int64_t pixels, int H, int W, int C, int cpad,
                                                        const T* __restrict__ dy, int64_t dy_ps, int dy_c0,
                                                        int64_t dy_pl, const float* __restrict__ dy_nchw, const T* __restrict__ pre,
                                                        int64_t pre_ps, const float* __restrict__ alpha, T* __restrict__ dyp,
                                                        float* __restrict__ part) {
  constexpr int VEC = TypeInfo<T>::VEC;
  const int G = cpad / VEC;                 // groups per pixel
  const int ppb = 256 / G;                  // pixels per block iteration
  const int tid = threadIdx.x;
  const int grp = tid % G, pl = tid / G;
  const bool active = pl < ppb;
  float sa[VEC], sb[VEC], al[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    sa[k] = 0.f; sb[k] = 0.f;
    const int c = grp * VEC + k;
    al[k] = (active && c < C) ? alpha[c] : 0.f;
  }
  const int64_t stride = (int64_t)gridDim.x * ppb;
  int64_t p0 = (int64_t)blockIdx.x * ppb + pl;
  const int64_t dy_cf = rdn_coff(dy_c0 + grp * VEC, dy_ps, dy_pl);   // channel offset of this thread's unit
  // NHWC fast path: 4 pixel iterations per trip with all 8 loads issued first
  // (unconditional, from a clamped valid pixel) -- the plain loop exposes one
  // HBM round trip per pixel, which is what the small level-2/3 passes pay
  if (active && !dy_nchw && ((dy_ps | dy_c0) % VEC) == 0) {
    for (; p0 < pixels; p0 += RDN_PRELU_PU * stride) {
      u32x4 gv[RDN_PRELU_PU], xv[RDN_PRELU_PU];
#pragma unroll
      for (int u = 0; u < RDN_PRELU_PU; ++u) {
        const int64_t pu = p0 + u * stride;
        const int64_t pc = pu < pixels ? pu : p0;
        gv[u] = *(const u32x4*)(dy + pc * dy_ps + dy_cf);
        xv[u] = *(const u32x4*)(pre + pc * pre_ps + grp * VEC);
      }
#pragma unroll
      for (int u = 0; u < RDN_PRELU_PU; ++u) {
        const int64_t pu = p0 + u * stride;
        if (pu >= pixels) break;
        float g[VEC], x[VEC], o[VEC];
        Unit16<T>::unpack(gv[u], g);
        Unit16<T>::unpack(xv[u], x);
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          const int c = grp * VEC + k;
          const bool valid = c < C;
          const bool pos = x[k] > 0.f;
          o[k] = valid ? (pos ? g[k] : al[k] * g[k]) : 0.f;
          if (valid && !pos) sa[k] += x[k] * g[k];
          sb[k] += o[k];
        }
        *(u32x4*)(dyp + pu * cpad + grp * VEC) = Unit16<T>::pack(o);
      }
    }
  }
  if (active) {
    for (int64_t p = p0; p < pixels; p += stride) {
      float g[VEC], x[VEC], o[VEC];
      if (dy_nchw) {
        const int64_t hw = (int64_t)H * W;
        const int64_t nimg = p / hw, r = p - nimg * hw;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          const int c = grp * VEC + k;
          g[k] = c < C ? dy_nchw[(nimg * C + c) * hw + r] : 0.f;
        }
      } else {
        const T* src = dy + p * dy_ps + dy_cf;
        if (((dy_ps | dy_c0) % VEC) == 0) {
          Unit16<T>::unpack(*(const u32x4*)src, g);
        } else {
#pragma unroll
          for (int k = 0; k < VEC; ++k) g[k] = to_f32(src[k]);
        }
      }
      Unit16<T>::unpack(*(const u32x4*)(pre + p * pre_ps + grp * VEC), x);
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        const int c = grp * VEC + k;
        const bool valid = c < C;
        const bool pos = x[k] > 0.f;
        o[k] = valid ? (pos ? g[k] : al[k] * g[k]) : 0.f;
        if (valid && !pos) sa[k] += x[k] * g[k];
        sb[k] += o[k];
      }
      *(u32x4*)(dyp + p * cpad + grp * VEC) = Unit16<T>::pack(o);
    }
  }
  // block reduction per channel: LDS [ppb][cpad] x 2, then one partial per
  // (block, channel) -- no atomics (one address per channel would serialise
  // thousands of blocks); prelu_finalize_kernel sums the partials.
  __shared__ float red[2][256 * 8];
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    red[0][tid * VEC + k] = active ? sa[k] : 0.f;
    red[1][tid * VEC + k] = active ? sb[k] : 0.f;
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    const int gg = c / VEC, kk = c % VEC;
    float a = 0.f, b = 0.f;
    for (int q = 0; q < ppb; ++q) {
      a += red[0][(q * G + gg) * VEC + kk];
      b += red[1][(q * G + gg) * VEC + kk];
    }
    part[(int64_t)blockIdx.x * 2 * C + c] = a;
    part[(int64_t)blockIdx.x * 2 * C + C + c] = b;
  }
}

// one block per (channel, {alpha, bias}): sum the per-block partials in a
// fixed order and add into the fp32 gradient
__global__ __launch_bounds__(256) void prelu_finalize_kernel(const float* __restrict__ part, int nblk, int C,
                                                             float* __restrict__ dalpha, float* __restrict__ dbias) {
  const int c = blockIdx.x % C, which = blockIdx.x / C;
  float s = 0.f;
  for (int b = threadIdx.x; b < nblk; b += 256) s += part[(int64_t)b * 2 * C + which * C + c];
  __shared__ float sh[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float* dst = which ? dbias : dalpha;
    if (dst) dst[c] += (sh[0] + sh[1]) + (sh[2] + sh[3]);
  }
}

// ------------------------------------------------------------------ interp / pack input
__global__ void interp_kernel(const float* __restrict__ clean, const float* __restrict__ noisy,
                              const float* __restrict__ tn, int batch, int64_t per, float* __restrict__ x) {
  const int64_t n4 = per / 4;
  const int64_t total = (int64_t)batch * n4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / n4);
    const float a = tn[b];
    const f32x4 c = ((const f32x4*)clean)[i], n = ((const f32x4*)noisy)[i];
    ((f32x4*)x)[i] = a * n + (1.f - a) * c;
  }
}

template <typename T>
__global__ void pack_input_kernel(const float* __restrict__ x, int N, int C, int H, int W, const float* __restrict__ t,
                                  int64_t t_sb, int64_t t_sh, int64_t t_sw, int has_t, T* __restrict__ out, int cpad) {
  const int64_t HW = (int64_t)H * W, P = (int64_t)N * HW;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = p / HW, r = p - n * HW;
    const int y = (int)(r / W), xx = (int)(r - (int64_t)y * W);
    T* o = out + p * cpad;
    for (int c = 0; c < cpad; ++c) {
      float v = 0.f;
      if (c < C) v = x[(n * C + c) * HW + r];
      else if (c == C && has_t) v = t[n * t_sb + y * t_sh + xx * t_sw];
      o[c] = from_f32<T>(v);
    }
  }
}

// ------------------------------------------------------------------ weight packing
__device__ __forceinline__ float pack_value(int mode, const float* __restrict__ w, int d0, int d1, int kh, int kw,
                                            int pad0, int pad1, int kc, int ck, int r, int k) {
  const int taps = kh * kw;
  if (mode == RDN_PACK_CONV_FWD) {  // P[a][tap*pad1 + b] = W[a][b][tap]  (chunked when ck > 0)
    int tap, b;
    if (ck > 0) { const int ch = k / kc, rem = k - ch * kc; tap = rem / ck; b = ch * ck + (rem - tap * ck); }
    else { tap = k / pad1; b = k - tap * pad1; }
    const int a = r;
    if (a < d0 && b < d1 && tap < taps) return w[((int64_t)a * d1 + b) * taps + tap];
  } else if (mode == RDN_PACK_CONV_DGRAD) {  // P[b][tap'*pad0 + a] = W[a][b][flip(tap')]
    int tp, a;
    if (ck > 0) { const int ch = k / kc, rem = k - ch * kc; tp = rem / ck; a = ch * ck + (rem - tp * ck); }
    else { tp = k / pad0; a = k - tp * pad0; }
    const int b = r;
    if (a < d0 && b < d1 && tp < taps) {
      const int ky = kh - 1 - tp / kw, kx = kw - 1 - tp % kw;
      return w[((int64_t)a * d1 + b) * taps + ky * kw + kx];
    }
  } else {  // GEMM_T: P[tap*d1 + b][a] = W[a][b][tap], K = pad0 >= d0
    const int tap = r / d1, b = r - tap * d1, a = k;
    if (tap < taps && a < d0) return w[((int64_t)a * d1 + b) * taps + tap];
  }
  return 0.f;
}

static inline int chunk_kc(int ck, int dtype) {
  const int sk = dtype == RDN_BF16 ? 64 : 32;
  return ck > 0 ? (9 * ck + sk - 1) / sk * sk : 0;
}

template <typename T>
__global__ void pack_weights_kernel(int mode, const float* __restrict__ w, int d0, int d1, int kh, int kw, int pad0,
                                    int pad1, T* __restrict__ out, int rows_pad, int kp, int ck, int kc) {
  const int64_t total = (int64_t)rows_pad * kp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / kp), k = (int)(i - (int64_t)r * kp);
    out[i] = from_f32<T>(pack_value(mode, w, d0, d1, kh, kw, pad0, pad1, kc, ck, r, k));
  }
}

// one thread = one 16-byte unit of packed output (kp is a multiple of 64, so a unit
// never straddles two rows); 32-bit index math (rows_pad * kp < 2^31 per pack).
// Measured per train step (r02): one element per thread with 64-bit divisions
// 133 us -> 72 us.  What remains is the gather: consecutive k of a packed row read
// weights 9 floats apart (OIHW -> [co][tap][ci]); a flattened index space over all
// packs (per-pack prefix in LDS) was slower (85 us).
template <typename T>
__global__ __launch_bounds__(256) void pack_weights_batched_kernel(const rdn_pack_item* __restrict__ items, int sk) {
  constexpr int VEC = TypeInfo<T>::VEC;
  const rdn_pack_item it = items[blockIdx.y];
  const int kc = it.ck > 0 ? (9 * it.ck + sk - 1) / sk * sk : 0;
  const int units = it.rows_pad * (it.kp / VEC);
  T* __restrict__ out = (T*)it.out;
  for (int u = blockIdx.x * 256 + threadIdx.x; u < units; u += gridDim.x * 256) {
    const int e = u * VEC, r = e / it.kp, k0 = e - r * it.kp;
    float v[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q)
      v[q] = pack_value(it.mode, it.w, it.d0, it.d1, it.kh, it.kw, it.pad0, it.pad1, kc, it.ck, r, k0 + q);
    *(u32x4*)(out + e) = Unit16<T>::pack(v);
  }
}

// ------------------------------------------------------------------ reductions
// two-level: per-block partials (fp32) then one block sums them.
__global__ __launch_bounds__(256) void charb_partial_kernel(const float* __restrict__ p, const float* __restrict__ t,
                                                            int64_t n, float eps2, float* __restrict__ part) {
  float sc = 0.f, sm = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float d = p[i] - t[i];
    sc += sqrtf(d * d + eps2);
    sm += d * d;
  }
  __shared__ float s[2][4];
  sc = wave_sum(sc);
  sm = wave_sum(sm);
  if ((threadIdx.x & 63) == 0) { s[0][threadIdx.x >> 6] = sc; s[1][threadIdx.x >> 6] = sm; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s[0][0] + s[0][1] + s[0][2] + s[0][3];
    part[2 * blockIdx.x + 1] = s[1][0] + s[1][1] + s[1][2] + s[1][3];
  }
}

__global__ __launch_bounds__(256) void charb_final_kernel(const float* __restrict__ part, int nb, int64_t n,
                                                          float* __restrict__ out) {
  double sc = 0.0, sm = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) { sc += part[2 * i]; sm += part[2 * i + 1]; }
  __shared__ double s[2][256];
  s[0][threadIdx.x] = sc; s[1][threadIdx.x] = sm;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) { s[0][threadIdx.x] += s[0][threadIdx.x + o]; s[1][threadIdx.x] += s[1][threadIdx.x + o]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) { out[0] = (float)(s[0][0] / (double)n); out[1] = (float)(s[1][0] / (double)n); }
}

__global__ void charb_bwd_kernel(const float* __restrict__ p, const float* __restrict__ t, int64_t n, float eps2,
                                 float wc, float wm, const float* __restrict__ gout, float* __restrict__ dp) {
  const float g = gout[0] / (float)n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float d = p[i] - t[i];
    dp[i] = g * (wc * (d / sqrtf(d * d + eps2)) + wm * 2.f * d);
  }
}

__global__ __launch_bounds__(256) void sq_partial_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ part) {
  float s = 0.f;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 v = ((const f32x4*)g)[i];
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += g[i] * g[i];
  __shared__ float sh[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// pre: a scale the caller has not applied to g yet (the data-parallel 1/world average,
// ddp.GradSync.defer_average): the norm is that of pre*g and out[1] carries pre; for a
// power-of-two pre both are exactly what scaling g first would give
__global__ __launch_bounds__(256) void sq_final_kernel(const float* __restrict__ part, int nb, float max_norm,
                                                       float pre, float* __restrict__ out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) s += part[i];
  __shared__ double sh[256];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float tot = (float)(sqrt(sh[0]) * (double)pre);
    out[0] = tot;
    const float coef = max_norm / (tot + 1e-6f);
    out[1] = pre * (coef < 1.f ? coef : 1.f);
  }
}

__global__ void scale_kernel(float* __restrict__ g, int64_t n, const float* __restrict__ coef) {
  const float c = coef[0];
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    ((f32x4*)g)[i] *= c;
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    g[i] *= c;
}

// torch.optim.Adam/AdamW single-tensor math (torch/optim/adam.py, _single_tensor_adam),
// with every scalar rounded to fp32 from the same double torch computes it in:
//   AdamW: p *= (1 - lr*wd) ; Adam: g += wd*p
//   m = lerp(m, g, 1-b1) ; v = v*b2 + (1-b2)*g*g
//   p += -(lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps),  bc_i = 1 - b_i^step
struct AdamScalars {
  float decay, wd, omb1, b2, omb2, step_size, bc2s, eps;
};
__host__ __device__ inline AdamScalars adam_scalars(double lr, double b1, double b2, double eps, double wd,
                                                    int decoupled, double step) {
  AdamScalars a;
  const double bc1 = 1.0 - pow(b1, step), bc2 = 1.0 - pow(b2, step);
  a.decay = decoupled ? (float)(1.0 - lr * wd) : 1.f;
  a.wd = decoupled ? 0.f : (float)wd;
  a.omb1 = (float)(1.0 - b1);
  a.b2 = (float)b2;
  a.omb2 = (float)(1.0 - b2);
  a.step_size = (float)(lr / bc1);
  a.bc2s = (float)sqrt(bc2);
  a.eps = (float)eps;
  return a;
}

// host_sc: the scalars of a host-known step; with step_dev != nullptr the step count
// is read from device memory (graph-replayable optimizer step) and the scalars are
// derived on the device in double, exactly as on the host
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, AdamScalars host_sc, const int64_t* __restrict__ step_dev,
                            double lr, double b1, double b2, double eps, double wd, int decoupled, float gs) {
  __shared__ AdamScalars sc_s;
  AdamScalars sc = host_sc;
  if (step_dev) {
    if (threadIdx.x == 0) sc_s = adam_scalars(lr, b1, b2, eps, wd, decoupled, (double)*step_dev);
    __syncthreads();
    sc = sc_s;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float pi = p[i], gi = g[i] * gs;
    pi *= sc.decay;
    gi += sc.wd * pi;
    const float mi = m[i] + (gi - m[i]) * sc.omb1;   // lerp form used by torch
    const float vi = v[i] * sc.b2 + sc.omb2 * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi += -sc.step_size * (mi / (sqrtf(vi) / sc.bc2s + sc.eps));
    p[i] = pi;
  }
}

__global__ void counter_inc_kernel(int64_t* c) { *c += 1; }

// the device's constant-rate wall clock when this kernel starts, by one lane (vector
// store): stream-ordered timestamps that a captured hipGraph replays (bench.py's
// exposed all-reduce time of the replayed data-parallel step)
__global__ void stamp_kernel(uint64_t* buf, int slot) {
  if (threadIdx.x == 0) buf[slot] = wall_clock64();
}

// x_tilde = (1-a)*f1 + a*y; x_tilde_prev = (1-ap)*f2 + ap*y; x = x - x_tilde + x_tilde_prev
// (diffusion_RDUnet.py:45-49), each product rounded separately as torch does.
__global__ void sampling_combine_kernel(float* __restrict__ x, const float* __restrict__ f1, const float* __restrict__ f2,
                                        const float* __restrict__ y, int64_t n, float c1, float a, float c2, float ap) {
#pragma clang fp contract(off)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float xt = c1 * f1[i] + a * y[i];
    const float xp = c2 * f2[i] + ap * y[i];
    x[i] = (x[i] - xt) + xp;
  }
}

template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ s, int N, int C, int H, int W, T* __restrict__ d,
                                    int64_t ps, int c0, int64_t pl, int acc) {
  const int64_t HW = (int64_t)H * W, total = (int64_t)N * C * HW;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / C;
    const int c = (int)(i - p * C);
    const int64_t n = p / HW, r = p - n * HW;
    T* const o = d + p * ps + rdn_coff(c0 + c, ps, pl);
    const float v = s[(n * C + c) * HW + r];
    *o = from_f32<T>(acc ? to_f32(*o) + v : v);
  }
}

template <typename T>
__global__ void nhwc_to_nchw_kernel(const T* __restrict__ s, int64_t ps, int c0, int64_t pl, int N, int C, int H, int W,
                                    float* __restrict__ d, int acc) {
  const int64_t HW = (int64_t)H * W, total = (int64_t)N * C * HW;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i % HW, nc = i / HW;
    const int c = (int)(nc % C);
    const int64_t n = nc / C;
    const float v = to_f32(s[(n * HW + r) * ps + rdn_coff(c0 + c, ps, pl)]);
    d[i] = acc ? d[i] + v : v;
  }
}

template <typename T>
__global__ void zero_slice_kernel(T* __restrict__ d, int64_t pixels, int64_t ps, int c0, int cols) {
  const int64_t total = pixels * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / cols;
    const int c = (int)(i - p * cols);
    d[p * ps + c0 + c] = from_f32<T>(0.f);
  }
}

}  // namespace

// ================================================================== C ABI
#define RDN_STREAM ((hipStream_t)stream)

static int prelu_blocks(int dtype, int64_t pixels, int cpad) {
  const int vec = dtype == RDN_BF16 ? 8 : 4;
  const int G = cpad / vec, ppb = 256 / G;
  return grid_for(pixels, ppb * 8, 1024);
}

extern "C" int32_t rdn_prelu_bwd_blocks(int32_t dtype, int64_t pixels, int32_t cpad) {
  return prelu_blocks(dtype, pixels, cpad);
}

extern "C" int64_t rdn_prelu_bwd_workspace_size(int32_t dtype, int64_t pixels, int32_t C, int32_t cpad) {
  return (int64_t)prelu_blocks(dtype, pixels, cpad) * 2 * C * (int64_t)sizeof(float);
}

extern "C" int rdn_prelu_bwd(int32_t dtype, int64_t pixels, int32_t n, int32_t h, int32_t w, int32_t C, int32_t cpad,
                             const void* dy, int64_t dy_ps, int32_t dy_c0, int64_t dy_pl, const float* dy_nchw, const void* pre,
                             int64_t pre_ps, const float* alpha, void* dyp, float* dalpha, float* dbias, float* ws,
                             void* stream) {
  const int vec = dtype == RDN_BF16 ? 8 : 4;
  if ((!dy && !dy_nchw) || !pre || !alpha || !dyp || !ws) { rdn_set_error("rdn_prelu_bwd: null pointer"); return RDN_E_ARG; }
  if (C <= 0 || cpad < C || cpad % vec || cpad / vec > 256 || pre_ps % vec || pixels != (int64_t)n * h * w) {
    rdn_set_error("rdn_prelu_bwd: bad shape C=%d cpad=%d pre_ps=%lld", C, cpad, (long long)pre_ps);
    return RDN_E_SHAPE;
  }
  const int blocks = prelu_blocks(dtype, pixels, cpad);
  if (dtype == RDN_BF16)
    prelu_bwd_kernel<bf16><<<blocks, 256, 0, RDN_STREAM>>>(pixels, h, w, C, cpad, (const bf16*)dy, dy_ps, dy_c0, dy_pl, dy_nchw,
                                                          (const bf16*)pre, pre_ps, alpha, (bf16*)dyp, ws);
  else
    prelu_bwd_kernel<float><<<blocks, 256, 0, RDN_STREAM>>>(pixels, h, w, C, cpad, (const float*)dy, dy_ps, dy_c0, dy_pl, dy_nchw,
                                                           (const float*)pre, pre_ps, alpha, (float*)dyp, ws);
  if (dalpha || dbias) prelu_finalize_kernel<<<2 * C, 256, 0, RDN_STREAM>>>(ws, blocks, C, dalpha, dbias);
  return rdn_check_launch("rdn_prelu_bwd");
}

extern "C" int rdn_interp(const float* clean, const float* noisy, const float* tnorm, int32_t batch, int64_t per,
                          float* x, void* stream) {
  if (!clean || !noisy || !tnorm || !x || per % 4 || ((uintptr_t)clean | (uintptr_t)noisy | (uintptr_t)x) & 15) {
    rdn_set_error("rdn_interp: bad arguments"); return RDN_E_ARG;
  }
  interp_kernel<<<grid_for(batch * per / 4, 256), 256, 0, RDN_STREAM>>>(clean, noisy, tnorm, batch, per, x);
  return rdn_check_launch("rdn_interp");
}

extern "C" int rdn_pack_input(int32_t dtype, const float* x, int32_t n, int32_t c, int32_t h, int32_t w, const float* t,
                              int64_t t_sb, int64_t t_sh, int64_t t_sw, int32_t has_t, void* out, int32_t cpad,
                              void* stream) {
  if (!x || !out || (has_t && !t) || cpad < c + (has_t ? 1 : 0)) { rdn_set_error("rdn_pack_input: bad arguments"); return RDN_E_ARG; }
  const int64_t P = (int64_t)n * h * w;
  if (dtype == RDN_BF16)
    pack_input_kernel<bf16><<<grid_for(P, 256), 256, 0, RDN_STREAM>>>(x, n, c, h, w, t, t_sb, t_sh, t_sw, has_t, (bf16*)out, cpad);
  else
    pack_input_kernel<float><<<grid_for(P, 256), 256, 0, RDN_STREAM>>>(x, n, c, h, w, t, t_sb, t_sh, t_sw, has_t, (float*)out, cpad);
  return rdn_check_launch("rdn_pack_input");
}

extern "C" int rdn_pack_weights_batched(const rdn_pack_item* items, int32_t n, int32_t dtype, void* stream) {
  if (!items || n <= 0 || n > 65535) { rdn_set_error("rdn_pack_weights_batched: bad arguments"); return RDN_E_ARG; }
  dim3 grid(96, n);   // 96 x 256 units per pass: the largest pack (level-3 conv_3) in ~8 passes
  if (dtype == RDN_BF16) pack_weights_batched_kernel<bf16><<<grid, 256, 0, RDN_STREAM>>>(items, 64);
  else pack_weights_batched_kernel<float><<<grid, 256, 0, RDN_STREAM>>>(items, 32);
  return rdn_check_launch("rdn_pack_weights_batched");
}

extern "C" int rdn_pack_weights(int32_t mode, int32_t dtype, const float* w, int32_t d0, int32_t d1, int32_t kh,
                                int32_t kw, int32_t pad0, int32_t pad1, void* out, int32_t rows_pad, int32_t kp,
                                int32_t ck, void* stream) {
  if (!w || !out || mode < 0 || mode > 2 || kp % 64 || rows_pad % 128) { rdn_set_error("rdn_pack_weights: bad arguments"); return RDN_E_ARG; }
  const int taps = kh * kw;
  const int kc = chunk_kc(ck, dtype);
  if (ck > 0) {
    const int kside = mode == RDN_PACK_CONV_FWD ? pad1 : pad0;
    if (taps != 9 || mode == RDN_PACK_GEMM_T || kside % ck || (kside / ck) * kc > kp) {
      rdn_set_error("rdn_pack_weights: chunked pack needs a 3x3 conv mode and kp >= %d", (kside / ck) * kc);
      return RDN_E_SHAPE;
    }
  } else if ((mode == RDN_PACK_CONV_FWD && (pad1 < d1 || rows_pad < d0 || taps * pad1 > kp)) ||
      (mode == RDN_PACK_CONV_DGRAD && (pad0 < d0 || rows_pad < d1 || taps * pad0 > kp)) ||
      (mode == RDN_PACK_GEMM_T && (pad0 < d0 || pad0 > kp || rows_pad < taps * d1))) {
    rdn_set_error("rdn_pack_weights: shape (mode=%d d0=%d d1=%d pad0=%d pad1=%d rows=%d kp=%d)", mode, d0, d1, pad0, pad1,
                  rows_pad, kp);
    return RDN_E_SHAPE;
  }
  const int64_t total = (int64_t)rows_pad * kp;
  if (dtype == RDN_BF16)
    pack_weights_kernel<bf16><<<grid_for(total, 256), 256, 0, RDN_STREAM>>>(mode, w, d0, d1, kh, kw, pad0, pad1, (bf16*)out, rows_pad, kp, ck, kc);
  else
    pack_weights_kernel<float><<<grid_for(total, 256), 256, 0, RDN_STREAM>>>(mode, w, d0, d1, kh, kw, pad0, pad1, (float*)out, rows_pad, kp, ck, kc);
  return rdn_check_launch("rdn_pack_weights");
}

static constexpr int kRedBlocks = 1024;
extern "C" int64_t rdn_reduce_workspace_size(int64_t) { return 2 * kRedBlocks * (int64_t)sizeof(float); }

extern "C" int rdn_charbonnier_fwd(const float* pred, const float* target, int64_t count, float eps, float* ws,
                                   float* out, void* stream) {
  if (!pred || !target || !ws || !out || count <= 0) { rdn_set_error("rdn_charbonnier_fwd: bad arguments"); return RDN_E_ARG; }
  const int nb = grid_for(count, 256 * 8, kRedBlocks);
  charb_partial_kernel<<<nb, 256, 0, RDN_STREAM>>>(pred, target, count, eps * eps, ws);
  charb_final_kernel<<<1, 256, 0, RDN_STREAM>>>(ws, nb, count, out);
  return rdn_check_launch("rdn_charbonnier_fwd");
}

extern "C" int rdn_charbonnier_bwd(const float* pred, const float* target, int64_t count, float eps, float wc, float wm,
                                   const float* gout, float* dpred, void* stream) {
  if (!pred || !target || !gout || !dpred || count <= 0) { rdn_set_error("rdn_charbonnier_bwd: bad arguments"); return RDN_E_ARG; }
  charb_bwd_kernel<<<grid_for(count, 256 * 4), 256, 0, RDN_STREAM>>>(pred, target, count, eps * eps, wc, wm, gout, dpred);
  return rdn_check_launch("rdn_charbonnier_bwd");
}

extern "C" int rdn_sqnorm_scaled(const float* g, int64_t count, float max_norm, float pre_scale, float* ws, float* out,
                                 void* stream) {
  if (!g || !ws || !out || count <= 0 || ((uintptr_t)g & 15) || !(pre_scale > 0.f)) {
    rdn_set_error("rdn_sqnorm: bad arguments");
    return RDN_E_ARG;
  }
  const int nb = grid_for(count, 256 * 16, kRedBlocks);
  sq_partial_kernel<<<nb, 256, 0, RDN_STREAM>>>(g, count, ws);
  sq_final_kernel<<<1, 256, 0, RDN_STREAM>>>(ws, nb, max_norm, pre_scale, out);
  return rdn_check_launch("rdn_sqnorm");
}

extern "C" int rdn_sqnorm(const float* g, int64_t count, float max_norm, float* ws, float* out, void* stream) {
  return rdn_sqnorm_scaled(g, count, max_norm, 1.f, ws, out, stream);
}

extern "C" int rdn_clip_scale(float* g, int64_t count, const float* coef, void* stream) {
  if (!g || !coef || count <= 0 || ((uintptr_t)g & 15)) { rdn_set_error("rdn_clip_scale: bad arguments"); return RDN_E_ARG; }
  scale_kernel<<<grid_for(count / 4 + 1, 256 * 4), 256, 0, RDN_STREAM>>>(g, count, coef);
  return rdn_check_launch("rdn_clip_scale");
}

extern "C" int rdn_adam_step(float* p, const float* g, float* m, float* v, int64_t count, double lr, double beta1,
                             double beta2, double eps, double wd, int32_t decoupled, int64_t step,
                             const int64_t* step_dev, float grad_scale, void* stream) {
  if (!p || !g || !m || !v || count <= 0 || (!step_dev && step < 1) || beta1 < 0 || beta1 >= 1 || beta2 < 0 ||
      beta2 >= 1) {
    rdn_set_error("rdn_adam_step: bad arguments");
    return RDN_E_ARG;
  }
  const AdamScalars sc = adam_scalars(lr, beta1, beta2, eps, wd, decoupled, (double)(step < 1 ? 1 : step));
  adam_kernel<<<grid_for(count, 256 * 4), 256, 0, RDN_STREAM>>>(p, g, m, v, count, sc, step_dev, lr, beta1, beta2, eps,
                                                               wd, decoupled, grad_scale);
  return rdn_check_launch("rdn_adam_step");
}

extern "C" int rdn_counter_inc(int64_t* counter, void* stream) {
  if (!counter) { rdn_set_error("rdn_counter_inc: null"); return RDN_E_ARG; }
  counter_inc_kernel<<<1, 1, 0, RDN_STREAM>>>(counter);
  return rdn_check_launch("rdn_counter_inc");
}

extern "C" int rdn_stamp(uint64_t* buf, int32_t slot, void* stream) {
  if (!buf || slot < 0) { rdn_set_error("rdn_stamp: bad arguments"); return RDN_E_ARG; }
  stamp_kernel<<<1, 64, 0, RDN_STREAM>>>(buf, slot);
  return rdn_check_launch("rdn_stamp");
}

extern "C" int64_t rdn_wall_clock_khz(void) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
      khz <= 0) {
    rdn_set_error("rdn_wall_clock_khz: no device clock rate");
    return RDN_E_LAUNCH;
  }
  return khz;
}

extern "C" int rdn_sampling_combine(float* x, const float* f1, const float* f2, const float* y, int64_t count, float c1,
                                    float a, float c2, float ap, void* stream) {
  if (!x || !f1 || !f2 || !y || count <= 0) { rdn_set_error("rdn_sampling_combine: bad arguments"); return RDN_E_ARG; }
  sampling_combine_kernel<<<grid_for(count, 256 * 4), 256, 0, RDN_STREAM>>>(x, f1, f2, y, count, c1, a, c2, ap);
  return rdn_check_launch("rdn_sampling_combine");
}

extern "C" int rdn_nchw_to_nhwc(int32_t dtype, const float* src, int32_t n, int32_t c, int32_t h, int32_t w, void* dst,
                                int64_t dst_ps, int32_t dst_c0, int64_t dst_pl, int32_t accumulate, void* stream) {
  if (!src || !dst || dst_ps <= 0) { rdn_set_error("rdn_nchw_to_nhwc: null / bad stride"); return RDN_E_ARG; }
  const int64_t total = (int64_t)n * c * h * w;
  if (dtype == RDN_BF16)
    nchw_to_nhwc_kernel<bf16><<<grid_for(total, 256 * 4), 256, 0, RDN_STREAM>>>(src, n, c, h, w, (bf16*)dst, dst_ps, dst_c0,
                                                                              dst_pl, accumulate);
  else
    nchw_to_nhwc_kernel<float><<<grid_for(total, 256 * 4), 256, 0, RDN_STREAM>>>(src, n, c, h, w, (float*)dst, dst_ps, dst_c0,
                                                                               dst_pl, accumulate);
  return rdn_check_launch("rdn_nchw_to_nhwc");
}

extern "C" int rdn_nhwc_to_nchw(int32_t dtype, const void* src, int64_t src_ps, int32_t src_c0, int64_t src_pl, int32_t n,
                                int32_t c, int32_t h, int32_t w, float* dst, int32_t accumulate, void* stream) {
  if (!src || !dst || src_ps <= 0) { rdn_set_error("rdn_nhwc_to_nchw: null / bad stride"); return RDN_E_ARG; }
  const int64_t total = (int64_t)n * c * h * w;
  if (dtype == RDN_BF16)
    nhwc_to_nchw_kernel<bf16><<<grid_for(total, 256 * 4), 256, 0, RDN_STREAM>>>((const bf16*)src, src_ps, src_c0, src_pl, n, c, h,
                                                                              w, dst, accumulate);
  else
    nhwc_to_nchw_kernel<float><<<grid_for(total, 256 * 4), 256, 0, RDN_STREAM>>>((const float*)src, src_ps, src_c0, src_pl, n, c,
                                                                               h, w, dst, accumulate);
  return rdn_check_launch("rdn_nhwc_to_nchw");
}

extern "C" int rdn_zero_slice(int32_t dtype, void* dst, int64_t pixels, int64_t ps, int32_t c0, int32_t cols, void* stream) {
  if (!dst || pixels < 0 || cols < 0) { rdn_set_error("rdn_zero_slice: bad arguments"); return RDN_E_ARG; }
  if (pixels == 0 || cols == 0) return RDN_OK;
  if (dtype == RDN_BF16)
    zero_slice_kernel<bf16><<<grid_for(pixels * cols, 256 * 4), 256, 0, RDN_STREAM>>>((bf16*)dst, pixels, ps, c0, cols);
  else
    zero_slice_kernel<float><<<grid_for(pixels * cols, 256 * 4), 256, 0, RDN_STREAM>>>((float*)dst, pixels, ps, c0, cols);
  return rdn_check_launch("rdn_zero_slice");
}

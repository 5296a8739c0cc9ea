// GPU data synthesis: one launch turns a batch of uint8
// patches resident in HBM into the (noisy, clean) fp32 NCHW pair in [-1, 1] that
// the reference's loaders produce per item on the host:
//
//   CustomDataset.__getitem__ (dataset_creation/custom_dataset.py:64-100):
//     crop -> float32 patch += N(0, sigma) (a float64 draw) -> np.clip(0, 255)
//     -> astype(uint8)                                          (:83-86)
//   CustomSIDD_Dataset.__getitem__ (dataset_creation/SIDD_dataset.py:74-97):
//     the same crop of a real (noisy, gt) pair, no synthetic noise
//   then the torchvision transforms (data_loader.py:35-46, SIDD_dataset.py:125-136),
//   drawn once per item and applied to both images (:89-95):
//     RandomHorizontalFlip -> RandomRotation(10) (PIL Image.rotate, NEAREST,
//     expand=False, fill 0) -> ToTensor (uint8 / 255) -> Normalize(0.5, 0.5).
//
// Rotation is Pillow's nearest-neighbour affine in 16.16 fixed point
// (Geometry.c affine_fixed, used whenever the corners fit in +-32768): the host
// passes the six integer coefficients, so output pixel (x, y) samples source
// ((a2 + y*a1 + x*a0) >> 16, (a5 + y*a4 + x*a3) >> 16) of the FLIPPED image, i.e.
// patch column P-1-xin when the flip fired.  Out-of-range samples take the fill
// value 0 in both images.
//
// Noise: either the caller's float64 draws (noise != NULL: the reference's own
// np.random.normal values, bit-exact reproduction), or a counter-based draw on
// the device: splitmix64(seed, element) -> two uniforms -> Box-Muller in double,
// z = sigma * sqrt(-2 ln u1) cos(2 pi u2) for element e = (py*P + px)*C + c of
// the unflipped source patch (oracle/synth_ref.py restates it in numpy).
//
// Thread = one output pixel of one item (all C channels); stores are coalesced
// per channel plane.  HBM-bound: P*P*C bytes gathered + 2 * 4*P*P*C written.
#include "rdn_common.h"

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// uniform in (0, 1) from the top 53 bits (oracle/weights.py _uniform01)
__device__ __forceinline__ double hash_u01(uint64_t key, uint64_t ctr) {
  const uint64_t h = splitmix64(splitmix64(ctr ^ key) + key);
  return ((double)(h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}

// ToTensor + Normalize(0.5, 0.5) with torch's CPU fp32 rounding: (q / 255 - 0.5) / 0.5
__device__ __forceinline__ float to_unit(int q) {
#pragma clang fp contract(off)
  const float v = (float)q / 255.0f;
  return (v - 0.5f) / 0.5f;
}

__global__ __launch_bounds__(256) void synth_kernel(const rdn_synth_item* __restrict__ items, int C, int P,
                                                    const uint8_t* __restrict__ clean_pool,
                                                    const uint8_t* __restrict__ noisy_pool,
                                                    const double* __restrict__ noise, float* __restrict__ out_noisy,
                                                    float* __restrict__ out_clean) {
#pragma clang fp contract(off)
  const int i = blockIdx.y;
  const int64_t pp = (int64_t)P * P;
  const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= pp) return;
  const rdn_synth_item it = items[i];
  const int y = (int)(pix / P), x = (int)(pix - (int64_t)y * P);
  int px = x, py = y;
  bool ok = true;
  if (it.rotate) {
    const int xx = it.affine[2] + y * it.affine[1] + x * it.affine[0];
    const int yy = it.affine[5] + y * it.affine[4] + x * it.affine[3];
    px = xx >> 16;   // arithmetic shift: floor, as Pillow's fixed-point path
    py = yy >> 16;
    ok = (unsigned)px < (unsigned)P && (unsigned)py < (unsigned)P;
  }
  if (it.flip) px = P - 1 - px;
  const int64_t src = (int64_t)py * it.row_stride + (int64_t)px * C;
  const int64_t eb = ((int64_t)py * P + px) * C;   // HWC element index in the unflipped patch
  float* const oc = out_clean + (int64_t)i * C * pp + pix;
  float* const on = out_noisy + (int64_t)i * C * pp + pix;
  for (int c = 0; c < C; ++c) {
    int qc = 0, qn = 0;
    if (ok) {
      qc = clean_pool[it.clean_off + src + c];
      if (noisy_pool) {
        qn = noisy_pool[it.noisy_off + src + c];
      } else {
        const int64_t e = eb + c;
        double z = 0.0;
        if (noise) {
          z = noise[(int64_t)i * pp * C + e];
        } else if (it.sigma != 0.f) {
          const double u1 = hash_u01(it.seed, 2 * (uint64_t)e), u2 = hash_u01(it.seed, 2 * (uint64_t)e + 1);
          z = (double)it.sigma * (sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
        }
        float v = (float)((double)qc + z);      // float32 += float64 (custom_dataset.py:85)
        v = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);   // np.clip(0, 255) (:86)
        qn = (int)v;                             // astype(uint8): truncation
      }
    }
    oc[c * pp] = to_unit(qc);
    on[c * pp] = to_unit(qn);
  }
}

}  // namespace

extern "C" int rdn_synth_batch(const rdn_synth_item* items, int32_t n, int32_t channels, int32_t patch,
                               const uint8_t* clean_pool, const uint8_t* noisy_pool, const double* noise,
                               float* out_noisy, float* out_clean, void* stream) {
  if (!items || !clean_pool || !out_noisy || !out_clean) { rdn_set_error("rdn_synth_batch: null pointer"); return RDN_E_ARG; }
  if (n <= 0 || n > 65535 || channels < 1 || channels > 4 || patch < 1 || patch > 8192) {
    rdn_set_error("rdn_synth_batch: bad shape n=%d channels=%d patch=%d", n, channels, patch);
    return RDN_E_SHAPE;
  }
  const int64_t pp = (int64_t)patch * patch;
  dim3 grid((unsigned)((pp + 255) / 256), (unsigned)n);
  synth_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(items, channels, patch, clean_pool, noisy_pool, noise, out_noisy,
                                                      out_clean);
  return rdn_check_launch("rdn_synth_batch");
}

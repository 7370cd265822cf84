// den_eval.hip -- the evaluation's image work outside the training step:
//
// * SSIM (loss_metric/metric.py:74-81, torchmetrics 0.6.2 functional.ssim with an 11 x 11 Gaussian
//   window of sigma 1.5, k1 = 0.01, k2 = 0.03): torchmetrics reflect-pads by 5, convolves, then crops
//   5 more from every side, so every kept window lies inside the image and the padding never enters
//   the result.  One thread per kept (channel, y, x): the five windowed moments in f32 (the products
//   p^2, t^2, p t rounded to f32 first, as torchmetrics forms them before its conv2d), the SSIM index
//   by torchmetrics' formula, and per image a deterministic f64 sum (block partials reduced in a
//   fixed order by sum_partials_f64_kernel).
// * PNG scanline unfiltering (host code): what libpng does inside the reference's cv2.imread
//   (data/datasets.py:508) for the 16-bit colour views PIL cannot decode losslessly.

namespace den {

constexpr int SSIM_BLOCK = 256, SSIM_SLICES = 128, SSIM_WIN = 11, SSIM_HALF = 5;

struct SsimArgs {
  int32_t C, H, W;
  float c1, c2;
  float win[SSIM_WIN * SSIM_WIN];
};

__global__ void __launch_bounds__(SSIM_BLOCK) ssim_kernel(SsimArgs A, const float* pred, const float* target,
                                                          double* part) {
  const int b = blockIdx.y, sl = blockIdx.x;
  const int Hk = A.H - 2 * SSIM_HALF, Wk = A.W - 2 * SSIM_HALF;
  const int64_t plane = (int64_t)A.H * A.W;
  const int64_t kept = (int64_t)A.C * Hk * Wk;
  const float* pb = pred + (int64_t)b * A.C * plane;
  const float* tb = target + (int64_t)b * A.C * plane;
  double acc = 0.0;
  for (int64_t k = (int64_t)sl * SSIM_BLOCK + threadIdx.x; k < kept; k += (int64_t)SSIM_SLICES * SSIM_BLOCK) {
    const int c = (int)(k / ((int64_t)Hk * Wk));
    const int r = (int)(k - (int64_t)c * Hk * Wk);
    const int y0 = r / Wk, x0 = r - (r / Wk) * Wk;  // window top-left = kept pixel - 5
    const float* p = pb + c * plane + (int64_t)y0 * A.W + x0;
    const float* t = tb + c * plane + (int64_t)y0 * A.W + x0;
    float mp = 0.f, mt = 0.f, epp = 0.f, ett = 0.f, ept = 0.f;
    for (int u = 0; u < SSIM_WIN; ++u) {
      for (int v = 0; v < SSIM_WIN; ++v) {
        const float w = A.win[u * SSIM_WIN + v];
        const float x = p[u * A.W + v], y = t[u * A.W + v];
        mp = fmaf(w, x, mp);
        mt = fmaf(w, y, mt);
        epp = fmaf(w, x * x, epp);
        ett = fmaf(w, y * y, ett);
        ept = fmaf(w, x * y, ept);
      }
    }
    const float mpp = mp * mp, mtt = mt * mt, mpt = mp * mt;
    const float spp = epp - mpp, stt = ett - mtt, spt = ept - mpt;
    const float upper = 2.f * spt + A.c2;
    const float lower = spp + stt + A.c2;
    acc += (double)(((2.f * mpt + A.c1) * upper) / ((mpp + mtt + A.c1) * lower));
  }
  __shared__ double s[SSIM_BLOCK];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int w = SSIM_BLOCK / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(int64_t)b * SSIM_SLICES + sl] = s[0];
}

// PNG filter types 0..4 (None, Sub, Up, Average, Paeth), bytewise with the left neighbour bpp bytes
// back; rows reconstructed in order.  Returns false on an unknown filter type.
static bool png_unfilter_host(int64_t height, int64_t row_bytes, int bpp, const uint8_t* in, uint8_t* out) {
  for (int64_t y = 0; y < height; ++y) {
    const uint8_t ft = in[y * (row_bytes + 1)];
    const uint8_t* f = in + y * (row_bytes + 1) + 1;
    uint8_t* o = out + y * row_bytes;
    const uint8_t* up = y > 0 ? out + (y - 1) * row_bytes : nullptr;
    for (int64_t i = 0; i < row_bytes; ++i) {
      const int a = i >= bpp ? o[i - bpp] : 0;
      const int b = up ? up[i] : 0;
      const int c = (up && i >= bpp) ? up[i - bpp] : 0;
      int pred;
      switch (ft) {
        case 0: pred = 0; break;
        case 1: pred = a; break;
        case 2: pred = b; break;
        case 3: pred = (a + b) >> 1; break;
        case 4: {
          const int p = a + b - c;
          const int pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
          pred = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
          break;
        }
        default: return false;
      }
      o[i] = (uint8_t)(f[i] + pred);
    }
  }
  return true;
}

}  // namespace den

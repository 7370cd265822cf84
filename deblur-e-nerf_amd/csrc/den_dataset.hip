// Raw-event preprocessing of the dataset loader (reference data/datasets.py):
//   * Event.queue_raw_events (:190-284): every raw event whose pixel saw an earlier raw event
//     (input order) with a different timestamp becomes a queued event [t_prev, t] with
//     num_pos = its own polarity, num_neg = 1 - num_pos; the others are dropped;
//   * Event.extract_max_refractory_period (:133-187): the minimum over pixels of the interval
//     between consecutive distinct timestamps -- the same predecessor relation (a pixel's last
//     kept timestamp always equals its immediately preceding raw event's), so it is the minimum
//     of t - t_prev over the queued events;
//   * Event.colorize_events (:287-328): the bayer channel of each queued event's pixel (its own
//     launch, as the reference's own step);
//   * Event.undistort_events (:331-364): OpenCV's undistortPoints (plumb_bob) /
//     fisheye::undistortPoints (equidistant) iterations, restated (OpenCV is not in the image:
//     parity unpinned).
//
// The reference walks the events in a Python loop with a per-pixel deque.  Here the predecessor
// relation comes from a stable LSD radix sort of the pixel keys (values = event indices, so
// equal keys keep input order): in sorted order an event's predecessor at its pixel is the entry
// before it when the keys agree.  Integer work only: every output is bit-exact by construction.
//
// Sort pass (8-bit digit): hist (per 4096-key tile, LDS atomics) -> per-digit scan over the
// tiles (one workgroup per digit) -> scatter (stable in-tile ranks by wave-wide digit matching:
// 8 ballots build each lane's same-digit mask, the lowest lane of a group bumps the wave's LDS
// counter for it, ranks = counter + popcount of the lower same-digit lanes; waves own
// contiguous quarters of the tile, so wave prefixes keep input order).

namespace den {

constexpr int QS_THREADS = 256;                // 4 waves
constexpr int QS_PER_WAVE_ITERS = 16;          // 16 x 64 keys per wave
constexpr int QS_TILE = QS_THREADS * QS_PER_WAVE_ITERS;  // 4096 keys per tile
constexpr int QS_RADIX = 256;

// pixel keys y * W + x and event indices; *status = 1 when a position lies outside the image
__global__ void queue_keys_kernel(int64_t n, int32_t H, int32_t W, const int64_t* __restrict__ position,
                                  uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, int32_t* status) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t x = position[2 * i], y = position[2 * i + 1];
  const bool ok = x >= 0 && x < W && y >= 0 && y < H;
  if (!ok) atomicOr(status, 1);
  keys[i] = ok ? (uint32_t)(y * W + x) : 0u;
  vals[i] = (uint32_t)i;
}

// counts[d * n_tiles + tile] = keys of digit d in the tile
__global__ void __launch_bounds__(QS_THREADS) radix_hist_kernel(int64_t n, int shift, const uint32_t* __restrict__ keys,
                                                                 uint32_t* __restrict__ counts, int64_t n_tiles) {
  __shared__ uint32_t h[QS_RADIX];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * QS_TILE;
#pragma unroll 4
  for (int k = 0; k < QS_PER_WAVE_ITERS; ++k) {
    const int64_t i = base + (int64_t)k * QS_THREADS + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 0xFF], 1u);
  }
  __syncthreads();
  counts[(int64_t)threadIdx.x * n_tiles + blockIdx.x] = h[threadIdx.x];
}

__device__ inline uint32_t block_excl_scan_u32(uint32_t v, uint32_t* total, uint32_t* s) {
  const int t = threadIdx.x;
  s[t] = v;
  __syncthreads();
  for (int off = 1; off < QS_THREADS; off <<= 1) {
    const uint32_t add = t >= off ? s[t - off] : 0u;
    __syncthreads();
    s[t] += add;
    __syncthreads();
  }
  const uint32_t incl = s[t];
  *total = s[QS_THREADS - 1];
  __syncthreads();
  return incl - v;
}

// one workgroup per digit: exclusive scan of its per-tile counts in place, digit total -> totals[d]
__global__ void __launch_bounds__(QS_THREADS) radix_scan_kernel(int64_t n_tiles, uint32_t* __restrict__ counts,
                                                                 uint32_t* __restrict__ totals) {
  __shared__ uint32_t s[QS_THREADS];
  uint32_t* c = counts + (int64_t)blockIdx.x * n_tiles;
  uint32_t carry = 0;
  for (int64_t b = 0; b < n_tiles; b += QS_THREADS) {
    const int64_t k = b + threadIdx.x;
    const uint32_t v = k < n_tiles ? c[k] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan_u32(v, &tot, s);
    if (k < n_tiles) c[k] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

__global__ void __launch_bounds__(QS_THREADS) radix_scatter_kernel(int64_t n, int shift, const uint32_t* __restrict__ keys,
                                                                    const uint32_t* __restrict__ vals,
                                                                    const uint32_t* __restrict__ counts,
                                                                    const uint32_t* __restrict__ totals, int64_t n_tiles,
                                                                    uint32_t* __restrict__ keys_out,
                                                                    uint32_t* __restrict__ vals_out) {
  __shared__ uint32_t wcount[4][QS_RADIX];
  __shared__ uint32_t base[4][QS_RADIX];
  __shared__ uint32_t s[QS_THREADS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int q = 0; q < 4; ++q) wcount[q][threadIdx.x] = 0;
  __syncthreads();
  const int64_t wbase = (int64_t)blockIdx.x * QS_TILE + (int64_t)w * (QS_TILE / 4);
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t key[QS_PER_WAVE_ITERS], val[QS_PER_WAVE_ITERS], rank[QS_PER_WAVE_ITERS];
#pragma unroll
  for (int k = 0; k < QS_PER_WAVE_ITERS; ++k) {
    const int64_t i = wbase + (int64_t)k * 64 + lane;
    const bool ok = i < n;
    key[k] = ok ? keys[i] : 0u;
    val[k] = ok ? vals[i] : 0u;
    const uint32_t d = (key[k] >> shift) & 0xFF;
    uint64_t m = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bb = __ballot((d >> b) & 1);
      m &= ((d >> b) & 1) ? bb : ~bb;
    }
    const int leader = __ffsll((unsigned long long)m) - 1;  // lowest lane of this digit group
    uint32_t b0 = 0;
    if (ok && lane == leader) {
      b0 = wcount[w][d];
      wcount[w][d] = b0 + (uint32_t)__popcll(m);
    }
    b0 = __shfl(b0, leader < 0 ? 0 : leader);
    rank[k] = b0 + (uint32_t)__popcll(m & lt);
  }
  __syncthreads();
  // digit d (thread d): exclusive prefix of the four waves' counts + the global base of this tile
  {
    const int d = threadIdx.x;
    uint32_t tot;
    const uint32_t dbase = block_excl_scan_u32(totals[d], &tot, s);
    uint32_t run = dbase + counts[(int64_t)d * n_tiles + blockIdx.x];
    for (int q = 0; q < 4; ++q) {
      base[q][d] = run;
      run += wcount[q][d];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < QS_PER_WAVE_ITERS; ++k) {
    const int64_t i = wbase + (int64_t)k * 64 + lane;
    if (i < n) {
      const uint32_t pos = base[w][(key[k] >> shift) & 0xFF] + rank[k];
      keys_out[pos] = key[k];
      vals_out[pos] = val[k];
    }
  }
}

// sorted position k: the event val[k] and its predecessor at the same pixel (val[k-1] when the
// keys agree) -> valid flag, start timestamp; block minimum of the valid intervals -> atomicMin
__global__ void queue_mark_kernel(int64_t n, const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                  const int64_t* __restrict__ ts, int32_t* __restrict__ valid,
                                  int64_t* __restrict__ start_ts, unsigned long long* __restrict__ min_interval_biased,
                                  unsigned long long* __restrict__ n_intervals) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t interval = INT64_MAX;
  int is_valid = 0;
  if (k < n) {
    const uint32_t i = vals[k];
    const int64_t t = ts[i];
    if (k > 0 && keys[k - 1] == keys[k]) {
      const int64_t tp = ts[vals[k - 1]];
      if (tp != t) {
        is_valid = 1;
        start_ts[i] = tp;
        interval = t - tp;
      }
    }
    valid[i] = is_valid;
  }
  // wave minimum (biased to unsigned order) + count, one atomic per wave
  unsigned long long v = (unsigned long long)interval ^ 0x8000000000000000ull;
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(v, off);
    v = o < v ? o : v;
  }
  const uint64_t cnt = __popcll(__ballot(is_valid));
  if ((threadIdx.x & 63) == 0 && cnt) {
    atomicMin(min_interval_biased, v);
    atomicAdd(n_intervals, (unsigned long long)cnt);
  }
}

struct QueueEmitArgs {
  int64_t n;
  const int64_t* position;
  const int64_t* ts;
  const uint8_t* polarity;
  const int32_t* valid;
  const int64_t* offsets;   // (n + 1) exclusive scan of valid
  const int64_t* start_tmp; // start timestamp per input event (valid ones)
  int64_t* out_position;
  int64_t* out_start_ts;
  int64_t* out_end_ts;
  int64_t* out_num_pos;
  int64_t* out_num_neg;
  const int32_t* status;
  const unsigned long long* min_biased;
  const unsigned long long* n_intervals;
  int64_t* out_count;       // (1): queued events, or -1 when a position is outside the image
  int64_t* out_min_interval;// (1): minimum interval (INT64_MAX when none)
  int64_t* out_n_intervals; // (1)
};

__global__ void queue_emit_kernel(QueueEmitArgs A) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    // stats only (den_max_refractory_period: no scan, offsets null): the count of intervals
    A.out_count[0] = A.status[0] ? -1 : (A.offsets ? A.offsets[A.n] : (int64_t)A.n_intervals[0]);
    if (A.out_min_interval) A.out_min_interval[0] = (int64_t)(A.min_biased[0] ^ 0x8000000000000000ull);
    if (A.out_n_intervals) A.out_n_intervals[0] = (int64_t)A.n_intervals[0];
  }
  if (i >= A.n || !A.valid[i] || !A.out_position) return;
  const int64_t o = A.offsets[i];
  const int64_t x = A.position[2 * i], y = A.position[2 * i + 1];
  A.out_position[2 * o] = x;
  A.out_position[2 * o + 1] = y;
  A.out_start_ts[o] = A.start_tmp[i];
  A.out_end_ts[o] = A.ts[i];
  const int64_t p = A.polarity[i] ? 1 : 0;
  A.out_num_pos[o] = p;
  A.out_num_neg[o] = 1 - p;
}

// colorize_events: channel of the bayer index (x odd) + 2 (y odd) -- top-left, top-right,
// bottom-left, bottom-right (datasets.py:307-327)
struct Bayer {
  int32_t ch[4];
};
__global__ void colorize_kernel(int64_t n, const int64_t* __restrict__ position, Bayer B, uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (uint8_t)B.ch[(int)(position[2 * i] & 1) + 2 * (int)(position[2 * i + 1] & 1)];
}

// ---- undistortion (OpenCV restated, double arithmetic on f32 inputs, f32 outputs)
struct UndistortArgs {
  int64_t n;
  int32_t model;     // 0 none (cast), 1 plumb_bob (k1 k2 p1 p2), 2 equidistant (k1..k4)
  double K[9];       // intrinsics (row-major 3x3), also the projection P (datasets.py:348-357 P=intrinsics)
  double D[4];
  const int64_t* position;
  float* out;
};

__global__ void undistort_kernel(UndistortArgs A) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n) return;
  // datasets.py:340-342: the positions are cast to the default dtype (f32) first
  const double u = (double)(float)A.position[2 * i], v = (double)(float)A.position[2 * i + 1];
  if (A.model == 0) {
    A.out[2 * i] = (float)u;
    A.out[2 * i + 1] = (float)v;
    return;
  }
  const double fx = A.K[0], fy = A.K[4], cx = A.K[2], cy = A.K[5];
  double x, y;
  bool ok = true;
  if (A.model == 1) {
    // cv::undistortPoints (cvUndistortPointsInternal), criteria COUNT 5
    x = (u - cx) * (1.0 / fx);
    y = (v - cy) * (1.0 / fy);
    const double x0 = x, y0 = y;
    const double k1 = A.D[0], k2 = A.D[1], p1 = A.D[2], p2 = A.D[3];
    for (int j = 0; j < 5; ++j) {
      const double r2 = x * x + y * y;
      const double icdist = 1.0 / (1.0 + (k2 * r2 + k1) * r2);
      if (icdist < 0) {
        x = (u - cx) * (1.0 / fx);
        y = (v - cy) * (1.0 / fy);
        break;
      }
      const double dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x);
      const double dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y;
      x = (x0 - dx) * icdist;
      y = (y0 - dy) * icdist;
    }
  } else {
    // cv::fisheye::undistortPoints, criteria MAX_ITER + EPS, 10, 1e-8
    const double pwx = (u - cx) / fx, pwy = (v - cy) / fy;
    double theta_d = sqrt(pwx * pwx + pwy * pwy);
    theta_d = fmin(fmax(-M_PI / 2, theta_d), M_PI / 2);
    bool converged = false;
    double theta = theta_d, scale = 0.0;
    if (fabs(theta_d) > 1e-8) {
      for (int j = 0; j < 10; ++j) {
        const double t2 = theta * theta, t4 = t2 * t2, t6 = t4 * t2, t8 = t6 * t2;
        const double a = A.D[0] * t2, b = A.D[1] * t4, c = A.D[2] * t6, d = A.D[3] * t8;
        const double fix = (theta * (1 + a + b + c + d) - theta_d) / (1 + 3 * a + 5 * b + 7 * c + 9 * d);
        theta = theta - fix;
        if (fabs(fix) < 1e-8) {
          converged = true;
          break;
        }
      }
      scale = tan(theta) / theta_d;
    } else {
      converged = true;
    }
    const bool flipped = (theta_d < 0 && theta > 0) || (theta_d > 0 && theta < 0);
    ok = converged && !flipped;
    x = pwx * scale;
    y = pwy * scale;
  }
  if (!ok) {
    A.out[2 * i] = -1000000.0f;
    A.out[2 * i + 1] = -1000000.0f;
    return;
  }
  // reprojection by P = K
  const double xx = A.K[0] * x + A.K[1] * y + A.K[2];
  const double yy = A.K[3] * x + A.K[4] * y + A.K[5];
  const double ww = 1.0 / (A.K[6] * x + A.K[7] * y + A.K[8]);
  A.out[2 * i] = (float)(xx * ww);
  A.out[2 * i + 1] = (float)(yy * ww);
}

}  // namespace den

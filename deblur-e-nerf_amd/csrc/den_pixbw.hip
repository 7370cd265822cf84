// den_pixbw.hip -- pixel-bandwidth sensor model (work in progress).
#include "den_device.h"

extern "C" {
int den_pixbw_blocks(int32_t N) { return (N + 255) / 256; }
int den_pixbw_sample_ts(int32_t, int32_t, const double*, const double*, double, double, double*, void*) { return 2; }
int den_pixbw_fwd(int32_t, int32_t, int32_t, const float*, const double*, const double*, const float*, const float*,
                  const double*, float*, float*, void*) { return 2; }
int den_pixbw_bwd(int32_t, int32_t, int32_t, const float*, const double*, const double*, const float*, const float*,
                  const double*, const float*, const float*, float*, float*, float*, void*) { return 2; }
}

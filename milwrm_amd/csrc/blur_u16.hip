// Fast fused log-normalise + Gaussian blur instances for uint16_t input (blur_mfma.h, blur.h).
#include "blur_mfma.h"

namespace mw {
template int launch_blur_fast<uint16_t>(const uint16_t*, int, int, int, const float*, float, const BlurTaps&,
                                    int, float*, hipStream_t);
}  // namespace mw

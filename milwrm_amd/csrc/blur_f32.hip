// Fast fused log-normalise + Gaussian blur instances for float input (blur_mfma.h, blur.h).
#include "blur_mfma.h"

namespace mw {
template int launch_blur_fast<float>(const float*, int, int, int, const float*, float, const BlurTaps&,
                                    int, float*, hipStream_t);
}  // namespace mw

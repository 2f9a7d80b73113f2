// Fused blur + subsample / label epilogue instances for uint16_t input (blur_mfma.h):
// a translation unit of their own so the blur kernels build in parallel.
#include "blur_mfma.h"

namespace mw {
template int launch_blur_epi<uint16_t>(const uint16_t*, int, int, int, const float*, float, const BlurTaps&, int,
                                   const BlurEpi&, int, hipStream_t);
}  // namespace mw

// Fused blur + subsample / label epilogue instances for float input (blur_mfma.h):
// a translation unit of their own so the blur kernels build in parallel.
#include "blur_mfma.h"

namespace mw {
template int launch_blur_epi<float>(const float*, int, int, int, const float*, float, const BlurTaps&, int,
                                   const BlurEpi&, int, hipStream_t);
}  // namespace mw

// fp32 instances of the blocked implicit-GEMM convolution (bconv_kernel.h):
// the fp32 training path (BASELINE config 2) on v_mfma_f32_16x16x4_f32.
#include "bconv_kernel.h"

namespace hcu {

int launch_bconv_f32(const GConvArgs &a, hipStream_t s) { BCONV_LAUNCH_BODY(float, "f32") }

}  // namespace hcu

/* batch_g2.hip -- aesgcm_batch_kernel instantiations for 2 lane(s) per record (batch_kernel.h) */
#include "batch_kernel.h"

namespace ptls_hip {

int launch_batch_g2(int rounds, bool open, int wg, unsigned grid, void *stream, const KernelArgs &a, bool aligned)
{
    return launch_batch_g<2>(rounds, open, wg, grid, static_cast<hipStream_t>(stream), a, aligned);
}

} // namespace ptls_hip

/* batch_g32.hip -- aesgcm_batch_kernel instantiations for 32 lanes per record (batch_kernel.h): two records per wave
 * task, the lanes' partial sums combined on the VALU.  For many keys with few records each (BASELINE configs[3]:
 * 64 records per key), where 16 lanes per record give a key run only 16 wave tasks for 12 waves. */
#include "batch_kernel.h"

namespace ptls_hip {

int launch_batch_g32(int rounds, bool open, int wg, unsigned grid, void *stream, const KernelArgs &a, bool aligned)
{
    return launch_batch_g<32>(rounds, open, wg, grid, static_cast<hipStream_t>(stream), a, aligned);
}

} // namespace ptls_hip

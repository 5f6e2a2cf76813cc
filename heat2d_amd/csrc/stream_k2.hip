// Instantiation of the streaming stencil for K = 2 fused time steps (see stream_kernel.hpp).
#include "stream_kernel.hpp"

namespace h2d {
template void launch_stream_k<2>(const StreamArgs&, bool, bool, hipStream_t);
template int stream_blocks_per_cu<2>(bool, bool);
}  // namespace h2d

// Instantiation of the streaming stencil for K = 5 fused time steps (see stream_kernel.hpp).
#include "stream_kernel.hpp"

namespace h2d {
template void launch_stream_k<5>(const StreamArgs&, bool, bool, hipStream_t);
template int stream_blocks_per_cu<5>(bool, bool);
}  // namespace h2d

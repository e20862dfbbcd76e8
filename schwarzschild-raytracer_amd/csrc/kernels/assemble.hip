// assemble.hip — device reassembly of gathered multi-GPU tiles (sr.h
// sr_assemble_blocks with on_device != 0). HBM-bound byte copy: one
// workgroup per (rank slot, row of the block, frame), 16-byte vector loads
// and stores along the row; each slot's frame block comes straight from
// its list entry, so no inverse map is built. Algorithmic bytes = 2 x the
// frame (read the gathered tiles once, write the frame once).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

__global__ __launch_bounds__(256) void sr_assemble_kernel(const uint8_t* __restrict__ stacked, size_t rank_stride,
                                                          size_t in_frame_stride, const int* __restrict__ lists,
                                                          int per, int height, int block_rows, size_t row_bytes,
                                                          uint8_t* __restrict__ out, size_t out_frame_stride) {
    const int slot = blockIdx.x / block_rows;  // r * per + s
    const int j = blockIdx.x % block_rows;
    const int f = blockIdx.y;
    const int b = lists[slot];
    if (b < 0) return;
    const int y = b * block_rows + j;
    if (y >= height) return;
    const int r = slot / per, s = slot % per;
    const uint8_t* src = stacked + (size_t)r * rank_stride + (size_t)f * in_frame_stride +
                         ((size_t)s * block_rows + j) * row_bytes;
    uint8_t* dst = out + (size_t)f * out_frame_stride + (size_t)y * row_bytes;
    if ((((uintptr_t)src | (uintptr_t)dst | row_bytes) & 15) == 0) {
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        for (size_t k = threadIdx.x; k < row_bytes / 16; k += blockDim.x) d4[k] = s4[k];
    } else {
        for (size_t k = threadIdx.x; k < row_bytes; k += blockDim.x) dst[k] = src[k];
    }
}

}  // namespace

extern "C" hipError_t sr_assemble_blocks_device(const uint8_t* stacked, size_t rank_stride, size_t in_frame_stride,
                                                const int* dev_lists, int world, int per, int height, int block_rows,
                                                size_t row_bytes, uint8_t* out, size_t out_frame_stride, int n_frames,
                                                hipStream_t stream) {
    const long long slots = (long long)world * per * block_rows;
    if (slots <= 0 || n_frames <= 0) return hipSuccess;
    if (slots > 0x7fffffffLL || n_frames > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sr_assemble_kernel, dim3((unsigned)slots, (unsigned)n_frames), dim3(256), 0, stream, stacked,
                       rank_stride, in_frame_stride, dev_lists, per, height, block_rows, row_bytes, out,
                       out_frame_stride);
    return hipGetLastError();
}

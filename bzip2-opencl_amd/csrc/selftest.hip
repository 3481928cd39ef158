// Device self-test of the cross-lane primitives in common.hpp (DPP / permlane
// moves and wave scans) against ds_bpermute shuffles and serial sums.
// Exposed as bz2mi_debug_selftest (tests/test_gpu.py runs it).
#include "common.hpp"
#include "kernels.hpp"

namespace bz2mi {

__global__ __launch_bounds__(64) void selftest_kernel(uint32_t* bad) {
    __shared__ uint32_t buf[64];
    const int lane = lane_id();
    for (int trial = 0; trial < 4; ++trial) {
        const uint32_t v = (uint32_t)lane * 0x9E3779B1u + 12345u * (uint32_t)(trial + 1);
        const uint32_t small = (v >> 20) & 1023u;
        if (xor_lanes<1>(v) != (uint32_t)__shfl_xor((int)v, 1)) atomicAdd(&bad[0], 1u);
        if (xor_lanes<2>(v) != (uint32_t)__shfl_xor((int)v, 2)) atomicAdd(&bad[1], 1u);
        if (xor_lanes<4>(v) != (uint32_t)__shfl_xor((int)v, 4)) atomicAdd(&bad[2], 1u);
        if (xor_lanes<8>(v) != (uint32_t)__shfl_xor((int)v, 8)) atomicAdd(&bad[3], 1u);
        if (xor_lanes<16>(v) != (uint32_t)__shfl_xor((int)v, 16)) atomicAdd(&bad[4], 1u);
        if (xor_lanes<32>(v) != (uint32_t)__shfl_xor((int)v, 32)) atomicAdd(&bad[5], 1u);
        const uint32_t prev = lane_prev(v, 77u);
        const uint32_t up = (uint32_t)__shfl_up((int)v, 1);  // (all lanes active)
        if (prev != (lane ? up : 77u)) atomicAdd(&bad[6], 1u);
        buf[lane] = small;
        __syncthreads();
        uint32_t ref = 0, refmax = 0;
        for (int k = 0; k <= lane; ++k) {
            ref += buf[k];
            refmax = buf[k] > refmax ? buf[k] : refmax;
        }
        __syncthreads();
        if (wave_incl_sum(small) != ref) atomicAdd(&bad[7], 1u);
        if (wave_incl_max(small) != refmax) atomicAdd(&bad[8], 1u);
        if (wave_sum(small) != (uint32_t)__shfl((int)wave_incl_sum(small), 63)) atomicAdd(&bad[9], 1u);
    }
}

int run_selftest(uint32_t* host_bad, int n) {
    uint32_t* d = nullptr;
    if (hipMalloc(&d, 16 * sizeof(uint32_t)) != hipSuccess) return -1;
    (void)hipMemset(d, 0, 16 * sizeof(uint32_t));
    hipLaunchKernelGGL(selftest_kernel, dim3(1), dim3(64), 0, 0, d);
    const hipError_t e = hipMemcpy(host_bad, d, sizeof(uint32_t) * (n < 16 ? n : 16), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? 10 : -1;
}

}  // namespace bz2mi

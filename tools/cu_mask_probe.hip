// Which (XCD, SE, CU) a CU-masked stream's workgroups land on: every workgroup records
// XCC_ID and HW_ID (s_getreg reads; vector stores only). tools/cu_mask_probe.py drives it.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void where_kernel(uint32_t* out)
{
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    // keep the workgroup resident for a while so the dispatcher spreads the grid
    float acc = threadIdx.x;
    for (int i = 0; i < 20000; ++i)
        acc = acc * 0.999f + 1.0f;
    if (threadIdx.x == 0)
    {
        out[2 * blockIdx.x]     = xcc;
        out[2 * blockIdx.x + 1] = hw + (acc < 0.0f ? 1u : 0u);
    }
}

extern "C" int probe_where(const uint32_t* mask, uint32_t words, int blocks, uint32_t* host_out)
{
    hipStream_t s = nullptr;
    if (words)
    {
        if (hipExtStreamCreateWithCUMask(&s, words, mask) != hipSuccess)
            return -1;
    }
    else if (hipStreamCreate(&s) != hipSuccess)
        return -1;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, sizeof(uint32_t) * 2 * blocks) != hipSuccess)
        return -2;
    hipLaunchKernelGGL(where_kernel, dim3(blocks), dim3(64), 0, s, d);
    if (hipStreamSynchronize(s) != hipSuccess)
        return -3;
    hipMemcpy(host_out, d, sizeof(uint32_t) * 2 * blocks, hipMemcpyDeviceToHost);
    hipFree(d);
    hipStreamDestroy(s);
    return 0;
}

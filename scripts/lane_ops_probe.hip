// Probe of the gfx950 lane-exchange instructions used by transpose64: prints,
// per lane, what v_permlane32_swap / v_permlane16_swap / DPP row_ror:8 /
// quad_perm return for x = lane, y = 100 + lane.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
    const unsigned x = threadIdx.x, y = 100 + threadIdx.x;
    const auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    const auto s = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    o[threadIdx.x * 8 + 0] = r[0];
    o[threadIdx.x * 8 + 1] = r[1];
    o[threadIdx.x * 8 + 2] = s[0];
    o[threadIdx.x * 8 + 3] = s[1];
    o[threadIdx.x * 8 + 4] = __builtin_amdgcn_update_dpp(0u, x, 0x128, 0xf, 0xf, false);  // row_ror:8
    o[threadIdx.x * 8 + 5] = __builtin_amdgcn_update_dpp(0u, x, 0x4e, 0xf, 0xf, false);   // quad_perm 2,3,0,1
    o[threadIdx.x * 8 + 6] = __builtin_amdgcn_update_dpp(0u, x, 0xb1, 0xf, 0xf, false);   // quad_perm 1,0,3,2
    o[threadIdx.x * 8 + 7] = __builtin_amdgcn_update_dpp(0u, x, 0x141, 0xf, 0xf, false);  // row_half_mirror
}
int main() {
    unsigned* d;
    if (hipMalloc(&d, 64 * 8 * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    unsigned h[64 * 8];
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    for (int l = 0; l < 64; ++l)
        std::printf("lane %2d: p32 %3u %3u  p16 %3u %3u  ror8 %2u  qp2301 %2u  qp1032 %2u  hmir %2u\n", l, h[l * 8],
                    h[l * 8 + 1], h[l * 8 + 2], h[l * 8 + 3], h[l * 8 + 4], h[l * 8 + 5], h[l * 8 + 6], h[l * 8 + 7]);
    return 0;
}

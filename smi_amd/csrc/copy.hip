// copy.hip -- several device-to-device copies in one kernel launch.
//
// The in-process transport (transport.cpp) moves every receive of a group
// with one launch instead of one hipMemcpyAsync per message: a K-step
// exchange of an interior rank is 8 messages per pass, and per-message host
// calls (copy + events) cost more host time than the pass itself
// (profiles/r03/).  Segments whose pointers or sizes are not 16-byte
// multiples go through hipMemcpyAsync.  Bulk point-to-point messages of the
// in-process transport (smi_send / smi_recv, hosts/bandwidth_benchmark) are
// copied by the same kernel.
#include "smi_internal.h"

namespace smi {

constexpr int kCopyMaxSegs = 16;
struct CopySegs {
    const uint4 *src[kCopyMaxSegs];
    uint4 *dst[kCopyMaxSegs];
    unsigned long long n16[kCopyMaxSegs];
    int first_block[kCopyMaxSegs + 1];
};

__global__ __launch_bounds__(256) void multicopy_kernel(CopySegs c, int nseg) {
    const int b = blockIdx.x;
    int seg = 0;
    for (int k = 1; k < nseg; ++k) seg += b >= c.first_block[k];
    const int b0 = seg == 0 ? 0 : c.first_block[seg];
    const int nb = c.first_block[seg + 1] - b0;
    const uint4 *src = c.src[seg];
    uint4 *dst = c.dst[seg];
    const unsigned long long n = c.n16[seg], S = (unsigned long long)nb * 256;
    unsigned long long i = (unsigned long long)(b - b0) * 256 + threadIdx.x;
    for (; i + 3 * S < n; i += 4 * S) {  // four loads in flight before the stores
        const uint4 a0 = src[i], a1 = src[i + S], a2 = src[i + 2 * S], a3 = src[i + 3 * S];
        dst[i] = a0;
        dst[i + S] = a1;
        dst[i + 2 * S] = a2;
        dst[i + 3 * S] = a3;
    }
    for (; i < n; i += S) dst[i] = src[i];
}

#ifdef SMI_LOOPBACK_REHEARSAL
// Rehearsal only: the same copies with the resource footprint of RCCL's
// rcclGenericKernel<4> on gfx950 (tools/rccl_footprint.py: 280 VGPRs incl.
// 32 AGPRs, 256-thread workgroups, 19,744 B of LDS), so that the exchange
// finds wave slots beside the interior sweep exactly as RCCL's kernel would.
// `blocks` plays RCCL's channel count; every block walks every segment.
__global__ __launch_bounds__(256) void heavycopy_kernel(CopySegs c, int nseg) {
    __shared__ uint4 lds[19744 / 16];
    asm volatile("; rccl footprint" ::: "v247", "a31");  // 248 + 32 = 280 registers, as rcclGenericKernel<4>
    lds[threadIdx.x] = make_uint4(threadIdx.x, 0, 0, 0);
    __syncthreads();
    const unsigned long long stride = (unsigned long long)gridDim.x * 256;
    for (int seg = 0; seg < nseg; ++seg) {
        const uint4 *src = c.src[seg];
        uint4 *dst = c.dst[seg];
        for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < c.n16[seg]; i += stride)
            dst[i] = src[i];
    }
    if (lds[(threadIdx.x + 1) & 255].x == 0xffffffffu) c.dst[0][0] = make_uint4(0, 0, 0, 0);  // keeps the LDS
}

int launch_heavy_copies(const void *const *src, void *const *dst, const size_t *bytes, int n, int blocks,
                        hipStream_t s) {
    CopySegs c{};
    int nseg = 0;
    for (int i = 0; i < n && nseg < kCopyMaxSegs; ++i) {
        if (bytes[i] == 0) continue;
        if (((uintptr_t)src[i] & 15u) || ((uintptr_t)dst[i] & 15u) || bytes[i] % 16) return SMI_ERR_INVALID_ARG;
        c.src[nseg] = reinterpret_cast<const uint4 *>(src[i]);
        c.dst[nseg] = reinterpret_cast<uint4 *>(dst[i]);
        c.n16[nseg] = bytes[i] / 16;
        ++nseg;
    }
    hipLaunchKernelGGL(heavycopy_kernel, dim3(std::max(1, blocks)), dim3(256), 0, s, c, nseg);
    SMI_HIP_CHECK(hipGetLastError());
    return SMI_SUCCESS;
}
#endif

int launch_copies(const void *const *src, void *const *dst, const size_t *bytes, int n, hipStream_t s) {
    CopySegs c{};
    int nseg = 0, blocks = 0;
    auto flush = [&]() -> int {
        if (nseg == 0) return SMI_SUCCESS;
        c.first_block[nseg] = blocks;
        hipLaunchKernelGGL(multicopy_kernel, dim3(blocks), dim3(256), 0, s, c, nseg);
        SMI_HIP_CHECK(hipGetLastError());
        nseg = blocks = 0;
        return SMI_SUCCESS;
    };
    for (int i = 0; i < n; ++i) {
        if (bytes[i] == 0) continue;
        const bool vec = ((uintptr_t)src[i] & 15u) == 0 && ((uintptr_t)dst[i] & 15u) == 0 && bytes[i] % 16 == 0;
        if (!vec) {
            SMI_HIP_CHECK(hipMemcpyAsync(dst[i], src[i], bytes[i], hipMemcpyDeviceToDevice, s));
            continue;
        }
        const size_t n16 = bytes[i] / 16;
        c.src[nseg] = reinterpret_cast<const uint4 *>(src[i]);
        c.dst[nseg] = reinterpret_cast<uint4 *>(dst[i]);
        c.n16[nseg] = n16;
        c.first_block[nseg] = blocks;
        // ~4 vectors per thread; a large message gets up to 8 workgroups per
        // CU (a halo of 16-32 KiB gets one or two)
        blocks += (int)std::min<size_t>(2048, std::max<size_t>(1, (n16 + 1023) / 1024));
        if (++nseg == kCopyMaxSegs) SMI_TRY(flush());
    }
    return flush();
}

}  // namespace smi

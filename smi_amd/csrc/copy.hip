// copy.hip -- several device-to-device copies in one kernel launch.
//
// The in-process transport (transport.cpp) moves every receive of a group
// with one launch instead of one hipMemcpyAsync per message: a K-step
// exchange of an interior rank is 8 messages per pass, and per-message host
// calls (copy + events) cost more host time than the pass itself
// (profiles/r03/).  Segments whose pointers or sizes are not 16-byte
// multiples go through hipMemcpyAsync.
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
    const unsigned long long n = c.n16[seg];
    for (unsigned long long i = (unsigned long long)(b - b0) * 256 + threadIdx.x; i < n; i += (unsigned long long)nb * 256)
        dst[i] = src[i];
}

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
        blocks += (int)std::min<size_t>(256, std::max<size_t>(1, (n16 + 1023) / 1024));  // ~4 vectors per thread
        if (++nseg == kCopyMaxSegs) SMI_TRY(flush());
    }
    return flush();
}

}  // namespace smi

// Diagnostic: which XCD (XCC_ID hardware register) each workgroup of a launch runs on, against the blockIdx % 8 rule
// the trace kernels' XCD placement assumes. Launches of 2048 and 32768 workgroups of 256 threads; each workgroup does
// a little arithmetic so that later workgroups are dispatched while earlier ones still run.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) k_xcc(unsigned *out, unsigned iters) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    float a = (float)threadIdx.x;
    for (unsigned i = 0; i < iters; ++i) a = a * 1.0001f + 0.5f;
    if (threadIdx.x == 0) out[blockIdx.x] = (x & 0xFu) | (a == -1.0f ? 16u : 0u);
}

int main() {
    for (unsigned n : {2048u, 32768u}) {
        for (unsigned iters : {0u, 20000u}) {
            unsigned *d;
            if (hipMalloc(&d, n * 4) != hipSuccess) return 1;
            k_xcc<<<n, 256>>>(d, iters);
            if (hipDeviceSynchronize() != hipSuccess) return 2;
            std::vector<unsigned> h(n);
            if (hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 3;
            unsigned match = 0, hist[8] = {0};
            for (unsigned b = 0; b < n; ++b) {
                match += (h[b] & 7u) == (b & 7u);
                hist[h[b] & 7u]++;
            }
            printf("blocks %u iters %u: xcc == blockIdx %% 8 for %u of %u; per-XCC counts", n, iters, match, n);
            for (unsigned k = 0; k < 8; ++k) printf(" %u", hist[k]);
            printf("\n");
            (void)hipFree(d);
        }
    }
    return 0;
}

// Repro probe for the round-1 anomaly "a stream-ordered hipMallocAsync staging buffer intermittently handed the kernel
// stale ray data after a pageable host copy" (vhx_trace_rays before bb24bbb). Mirrors the old call sequence: per call,
// hipMallocAsync(staging) -> hipMemcpyAsync(staging <- pageable host, H2D) -> kernel reads staging -> D2H of the
// output -> hipStreamSynchronize -> hipFreeAsync(staging) -> hipStreamSynchronize. Each call stamps its host data with
// the call number; the kernel counts words that do not carry the stamp (stale data). Mode 0: hipMallocAsync staging
// (the old code); 1: a context-owned hipMalloc buffer grown on demand (the fix); 2: mode 0 with the stream switched
// between two streams every call (a caller's set_stream); 3: mode 0 on the legacy null stream.
// Build: hipcc --offload-arch=gfx950 -O2 mallocasync_stale.hip -o mallocasync_stale; run: ./mallocasync_stale MODE CALLS
// (the ROCm 7.2 runtime of /opt/rocm); or -DAS_LIB -shared -fPIC -o libmallocasync_stale.so, loaded by
// mallocasync_stale.py after torch (torch's own HIP runtime, the one libvhx runs on under Python).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
            return 2;                                                                              \
        }                                                                                          \
    } while (0)

__global__ void k_check(const unsigned *in, unsigned long long n, unsigned stamp, unsigned *out,
                        unsigned *bad) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned v = in[i];
    out[i] = v;
    if (v != (stamp ^ (unsigned)(i * 2654435761u))) atomicAdd(bad, 1u);  // a vector atomic on global memory
}

extern "C" int anomaly_run(int mode, int calls) {
    hipStream_t s[2];
    CK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking));
    unsigned *bad, *out = nullptr, *own = nullptr;
    size_t out_cap = 0, own_cap = 0;
    CK(hipMalloc(&bad, 4));
    CK(hipMemset(bad, 0, 4));
    unsigned long long stale_calls = 0, words = 0;
    unsigned prev_bad = 0;
    for (int k = 1; k <= calls; ++k) {
        // ray batches of 6 floats per ray, 1 .. ~60 k rays, sizes varying from call to call
        const unsigned long long n = 6ull * (1 + (unsigned long long)(k * 7919u) % 60000u);
        std::vector<unsigned> host(n), back(n);  // pageable
        for (unsigned long long i = 0; i < n; ++i) host[i] = (unsigned)k ^ (unsigned)(i * 2654435761u);
        hipStream_t st = mode == 3 ? (hipStream_t)0 : s[mode == 2 ? (k & 1) : 0];
        if (out_cap < n * 4) {  // the context's scratch output (ensure(): hipFree + hipMalloc when it grows)
            if (out) CK(hipFree(out));
            CK(hipMalloc(&out, n * 4));
            out_cap = n * 4;
        }
        unsigned *staging = nullptr;
        if (mode == 1) {
            if (own_cap < n * 4) {
                if (own) CK(hipFree(own));
                CK(hipMalloc(&own, n * 4));
                own_cap = n * 4;
            }
            staging = own;
        } else {
            CK(hipMallocAsync((void **)&staging, n * 4, st));
        }
        CK(hipMemcpyAsync(staging, host.data(), n * 4, hipMemcpyHostToDevice, st));
        k_check<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(staging, n, (unsigned)k, out, bad);
        CK(hipGetLastError());
        CK(hipMemcpyAsync(back.data(), out, n * 4, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        if (mode != 1) {
            CK(hipFreeAsync(staging, st));
            CK(hipStreamSynchronize(st));
        }
        unsigned b = 0;
        CK(hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost));
        if (b != prev_bad) {
            ++stale_calls;
            words += b - prev_bad;
            if (stale_calls <= 5) fprintf(stderr, "call %d: %u stale words of %llu\n", k, b - prev_bad, n);
            prev_bad = b;
        }
    }
    printf("mode %d: %d calls, %llu with stale staging data (%llu words)\n", mode, calls, stale_calls, words);
    fflush(stdout);
    return stale_calls ? 1 : 0;
}

#ifndef AS_LIB
int main(int argc, char **argv) { return anomaly_run(argc > 1 ? atoi(argv[1]) : 0, argc > 2 ? atoi(argv[2]) : 2000); }
#endif

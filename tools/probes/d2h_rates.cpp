// Host-link rates that bound the frontier spill: pinned allocation cost,
// device->host into pinned and pageable memory, device->device shift.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
    const size_t GB = 1ull << 30, N = 8 * GB;
    void *d, *d2, *h, *p;
    CK(hipMalloc(&d, N));
    CK(hipMalloc(&d2, N));
    CK(hipMemset(d, 1, N));
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    double t = now();
    CK(hipHostMalloc(&h, N, hipHostMallocDefault));
    printf("{\"hipHostMalloc_GBps\": %.2f}\n", N / (now() - t) / 1e9);
    for (int r = 0; r < 2; ++r) {
        t = now();
        CK(hipMemcpyAsync(h, d, N, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        printf("{\"d2h_pinned_GBps\": %.2f}\n", N / (now() - t) / 1e9);
    }
    t = now();
    p = malloc(N);
    CK(hipMemcpy(p, d, N, hipMemcpyDeviceToHost));
    printf("{\"d2h_pageable_fresh_GBps\": %.2f}\n", N / (now() - t) / 1e9);
    t = now();
    CK(hipMemcpy(p, d, N, hipMemcpyDeviceToHost));
    printf("{\"d2h_pageable_touched_GBps\": %.2f}\n", N / (now() - t) / 1e9);
    t = now();
    CK(hipHostRegister(p, N, hipHostRegisterDefault));
    printf("{\"hipHostRegister_GBps\": %.2f}\n", N / (now() - t) / 1e9);
    t = now();
    CK(hipMemcpyAsync(p, d, N, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    printf("{\"d2h_registered_GBps\": %.2f}\n", N / (now() - t) / 1e9);
    CK(hipHostUnregister(p));
    t = now();
    CK(hipMemcpyAsync(d2, d, N, hipMemcpyDeviceToDevice, s));
    CK(hipStreamSynchronize(s));
    printf("{\"d2d_GBps\": %.2f}\n", N / (now() - t) / 1e9);
    // two streams: half each (two copy engines?)
    t = now();
    CK(hipMemcpyAsync(h, d, N / 2, hipMemcpyDeviceToHost, s));
    CK(hipMemcpyAsync((char*)h + N / 2, (char*)d + N / 2, N / 2, hipMemcpyDeviceToHost, s2));
    CK(hipStreamSynchronize(s));
    CK(hipStreamSynchronize(s2));
    printf("{\"d2h_pinned_2streams_GBps\": %.2f}\n", N / (now() - t) / 1e9);
    free(p);
    CK(hipHostFree(h));
    return 0;
}

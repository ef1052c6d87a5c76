// Host-link bandwidth probe: device -> page-locked host copies of one 1080p framebuffer (24.9 MB) by
// SDMA (1, 2, 4 streams splitting the buffer) and by a copy kernel storing to host-mapped memory.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
typedef float v4 __attribute__((ext_vector_type(4)));
__global__ void k_copy(const v4* __restrict__ s, v4* d, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(s[i], d + i);
}
__global__ void k_copy_plain(const v4* __restrict__ s, v4* d, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        d[i] = s[i];
}
int main() {
    const size_t bytes = 1920ull * 1080 * 12;
    void *d = nullptr, *h = nullptr, *hd = nullptr;
    hipMalloc(&d, bytes);
    hipMemset(d, 1, bytes);
    hipHostMalloc(&h, bytes, hipHostMallocDefault);
    hipHostGetDevicePointer(&hd, h, 0);
    hipStream_t st[4];
    for (auto& s : st) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    auto time = [&](auto fn, const char* name) {
        for (int i = 0; i < 3; ++i) fn();
        hipDeviceSynchronize();
        const int n = 20;
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < n; ++i) fn();
        hipDeviceSynchronize();
        double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / n;
        std::printf("%-34s %.3f ms  %.1f GB/s\n", name, s * 1e3, bytes / s / 1e9);
    };
    for (int k : {1, 2, 4}) {
        char nm[64];
        std::snprintf(nm, sizeof nm, "SDMA hipMemcpyAsync x%d streams", k);
        time([&] {
            const size_t part = bytes / k;
            for (int i = 0; i < k; ++i)
                hipMemcpyAsync((char*)h + i * part, (char*)d + i * part, i == k - 1 ? bytes - i * part : part,
                               hipMemcpyDeviceToHost, st[i]);
        }, nm);
    }
    for (int g : {64, 256, 1024}) {
        char nm[64];
        std::snprintf(nm, sizeof nm, "kernel nontemporal, %d WGs", g);
        time([&] { k_copy<<<g, 256, 0, st[0]>>>((const v4*)d, (v4*)hd, bytes / 16); }, nm);
        std::snprintf(nm, sizeof nm, "kernel plain store, %d WGs", g);
        time([&] { k_copy_plain<<<g, 256, 0, st[0]>>>((const v4*)d, (v4*)hd, bytes / 16); }, nm);
    }
    std::printf("device->device hipMemcpy for reference:\n");
    void* d2 = nullptr;
    hipMalloc(&d2, bytes);
    time([&] { hipMemcpyAsync(d2, d, bytes, hipMemcpyDeviceToDevice, st[0]); }, "D2D");
    return 0;
}

// Per-call latency floor of the small-call host path: what one empty launch
// plus a wait costs on this box (hipStreamSynchronize against a spin on
// hipStreamQuery), next to rs_encode_parity / rs_decode_missing of one 4+2
// stripe from pageable host buffers, 1000 B and 4 KiB shards.
//   hipcc -O2 --offload-arch=gfx950 -Iinclude tools/latency_probe.hip \
//     -Ljava-reed-solomon-distributed-file-system_amd/lib -lrsamd \
//     -Wl,-rpath,'$ORIGIN/../../java-reed-solomon-distributed-file-system_amd/lib' -o tools/bin/latency_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rs_amd.h"

__global__ void empty_kernel(int *p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static double per_call_us(F &&f, int reps = 2000) {
    for (int i = 0; i < 50; ++i) f();
    const double t0 = now_us();
    for (int i = 0; i < reps; ++i) f();
    return (now_us() - t0) / reps;
}

int main() {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    int *flag = nullptr;
    if (hipMalloc(&flag, 4) != hipSuccess) return 1;
    std::printf("launch + hipStreamSynchronize      %7.1f us\n", per_call_us([&] {
                    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, flag);
                    (void)hipStreamSynchronize(s);
                }));
    std::printf("launch + spin on hipStreamQuery    %7.1f us\n", per_call_us([&] {
                    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, flag);
                    while (hipStreamQuery(s) == hipErrorNotReady) {
                    }
                }));
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return 1;
    std::printf("launch + event + spin on query     %7.1f us\n", per_call_us([&] {
                    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, flag);
                    (void)hipEventRecord(ev, s);
                    while (hipEventQuery(ev) == hipErrorNotReady) {
                    }
                }));
    std::printf("hipMemcpyAsync 4 KiB H2D + sync    %7.1f us\n", [&] {
        std::vector<uint8_t> h(4096, 1);
        return per_call_us([&] {
            (void)hipMemcpyAsync(flag, h.data(), 4, hipMemcpyHostToDevice, s);
            (void)hipStreamSynchronize(s);
        });
    }());
    rs_codec *c = nullptr;
    if (rs_codec_create(4, 2, &c)) return 1;
    for (int S : {1000, 4096, 65536}) {
        std::vector<std::vector<uint8_t>> sh(6, std::vector<uint8_t>(S));
        for (int i = 0; i < 4; ++i)
            for (int b = 0; b < S; ++b) sh[i][b] = uint8_t(b * 7 + i);
        std::vector<uint8_t *> p(6);
        std::vector<int64_t> len(6, S);
        for (int i = 0; i < 6; ++i) p[i] = sh[i].data();
        std::printf("rs_encode_parity 4+2 x %6d B   %7.1f us\n", S,
                    per_call_us([&] { (void)rs_encode_parity(c, p.data(), 6, len.data(), 0, S); }, 1000));
        const uint8_t present[6] = {0, 1, 1, 1, 1, 0};
        std::printf("rs_decode_missing {0,5} x %6d B %7.1f us\n", S,
                    per_call_us([&] { (void)rs_decode_missing(c, p.data(), 6, len.data(), present, 0, S); }, 1000));
    }
    rs_codec_destroy(c);
    rs_thread_release();
    return 0;
}

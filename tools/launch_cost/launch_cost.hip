// Host cost of one hipLaunchKernelGGL by kernel shape (kernarg size, scratch, static LDS):
// hipcc --offload-arch=gfx950 -O2 launch_cost.hip -o launch_cost && ./launch_cost
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Big { double d[360]; };  // 2880 B, about k_trace's kernarg
template <int N> struct Arr { double d[N]; };
template <int N>
__global__ void k_arr(Arr<N> a, double* p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0) *p = a.d[N - 1] + a.d[0];
}
// a kernarg of N doubles: launch cost, and whether the last word arrives intact
template <int N>
void arr_probe(hipStream_t s, double* d_out) {
    Arr<N> a{};
    for (int i = 0; i < N; ++i) a.d[i] = i;
    hipError_t e = hipSuccess;
    const double us = per_launch_us(s, [&] { hipLaunchKernelGGL(k_arr<N>, dim3(256), dim3(512), 0, s, a, nullptr); e = hipGetLastError(); });
    hipLaunchKernelGGL(k_arr<N>, dim3(1), dim3(64), 0, s, a, d_out);
    double h = -1;
    (void)hipMemcpy(&h, d_out, 8, hipMemcpyDeviceToHost);
    printf("kernarg %6zu B: %.2f us, %s, last+first = %.0f (want %d)\n", sizeof(a), us, hipGetErrorString(e), h, N - 1);
}
__global__ void k_small(int* p) { if (p && threadIdx.x == 1000) *p = 1; }
__global__ void k_big(Big b, int* p) { if (p && threadIdx.x == 1000) *p = (int)b.d[threadIdx.x % 360]; }
__global__ void k_scratch(int* p, int n) {
    volatile int a[24];
    for (int i = 0; i < 24; ++i) a[i] = i * n;
    if (p && threadIdx.x == 1000) *p = a[n % 24];
}
__global__ void k_lds(int* p) {
    __shared__ double s[9800];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (p && threadIdx.x == 1000) *p = (int)s[(threadIdx.x + 1) % 512];
}

template <class F>
double per_launch_us(hipStream_t s, F launch) {
    for (int i = 0; i < 50; ++i) launch();
    (void)hipStreamSynchronize(s);
    const int n = 2000;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) {
        launch();
        if (i % 4 == 3) (void)hipStreamSynchronize(s);  // keep the queue short, like frames in flight
    }
    auto t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(s);
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    Big b{};
    printf("small %.2f us\n", per_launch_us(s, [&] { hipLaunchKernelGGL(k_small, dim3(256), dim3(512), 0, s, nullptr); }));
    printf("big-kernarg %.2f us\n", per_launch_us(s, [&] { hipLaunchKernelGGL(k_big, dim3(256), dim3(512), 0, s, b, nullptr); }));
    printf("scratch %.2f us\n", per_launch_us(s, [&] { hipLaunchKernelGGL(k_scratch, dim3(256), dim3(512), 0, s, nullptr, 3); }));
    printf("lds78k %.2f us\n", per_launch_us(s, [&] { hipLaunchKernelGGL(k_lds, dim3(256), dim3(512), 0, s, nullptr); }));
    printf("small %.2f us\n", per_launch_us(s, [&] { hipLaunchKernelGGL(k_small, dim3(256), dim3(512), 0, s, nullptr); }));
    // a frame group's batch as one graph (stage, trace, pack, unpack): one hipGraphLaunch
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    hipLaunchKernelGGL(k_small, dim3(1), dim3(256), 0, s, nullptr);
    hipLaunchKernelGGL(k_big, dim3(256), dim3(512), 0, s, b, nullptr);
    hipLaunchKernelGGL(k_small, dim3(256), dim3(512), 0, s, nullptr);
    hipLaunchKernelGGL(k_small, dim3(256), dim3(512), 0, s, nullptr);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    printf("graph-of-4 %.2f us\n", per_launch_us(s, [&] { (void)hipGraphLaunch(ge, s); }));
    printf("4-separate %.2f us\n", per_launch_us(s, [&] {
        hipLaunchKernelGGL(k_small, dim3(1), dim3(256), 0, s, nullptr);
        hipLaunchKernelGGL(k_big, dim3(256), dim3(512), 0, s, b, nullptr);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(512), 0, s, nullptr);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(512), 0, s, nullptr);
    }));
    printf("scratch+3 %.2f us\n", per_launch_us(s, [&] {
        hipLaunchKernelGGL(k_small, dim3(1), dim3(256), 0, s, nullptr);
        hipLaunchKernelGGL(k_scratch, dim3(256), dim3(512), 0, s, nullptr, 3);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(512), 0, s, nullptr);
        hipLaunchKernelGGL(k_small, dim3(256), dim3(512), 0, s, nullptr);
    }));
    double* d_out = nullptr;
    (void)hipMalloc((void**)&d_out, 8);
    arr_probe<512>(s, d_out);
    arr_probe<1024>(s, d_out);
    arr_probe<2048>(s, d_out);
    arr_probe<3584>(s, d_out);
    arr_probe<4096>(s, d_out);
    arr_probe<6144>(s, d_out);
    arr_probe<8192>(s, d_out);
    return 0;
}

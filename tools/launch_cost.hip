// Host-side enqueue cost of the calls launch_batch makes (kernel launches with small and
// with PairConst-sized arguments, event records, cross-stream waits, async copies), on
// two non-blocking streams as the engine uses them.  Build + run:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/launch_cost.hip -o tools/launch_cost
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                                          \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            std::printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__);                                    \
            std::exit(1);                                                                                              \
        }                                                                                                              \
    } while (0)

struct Small { int a[4]; };
struct Big { double a[85]; }; // 680 bytes, like PairConst + PairData

__global__ void k_small(Small s, int *out) { if (threadIdx.x == 0 && s.a[0] < 0) out[0] = 1; }
__global__ void k_big(Big b, int *out) { if (threadIdx.x == 0 && b.a[0] < 0) out[0] = 1; }

using Clock = std::chrono::steady_clock;
static double us(Clock::time_point a) { return std::chrono::duration<double, std::micro>(Clock::now() - a).count(); }

int main() {
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    int *d;
    CK(hipMalloc(&d, 1 << 22));
    int *h;
    CK(hipHostMalloc(&h, 1 << 22, hipHostMallocDefault));
    hipEvent_t ev[8];
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    Small sm{};
    Big bg{};
    const int N = 2000;
    for (int rep = 0; rep < 3; ++rep) {
        double t_small = 0, t_big = 0, t_rec = 0, t_wait = 0, t_h2d = 0, t_h2d_big = 0, t_d2h = 0, t_grid = 0;
        for (int i = 0; i < N; ++i) {
            auto t = Clock::now();
            k_small<<<1, 64, 0, s0>>>(sm, d);
            t_small += us(t);
            t = Clock::now();
            k_big<<<1, 64, 0, s0>>>(bg, d);
            t_big += us(t);
            t = Clock::now();
            k_big<<<4096, 64, 0, s0>>>(bg, d);
            t_grid += us(t);
            t = Clock::now();
            CK(hipEventRecord(ev[i & 7], s0));
            t_rec += us(t);
            t = Clock::now();
            CK(hipStreamWaitEvent(s1, ev[i & 7], 0));
            t_wait += us(t);
            t = Clock::now();
            CK(hipMemcpyAsync(d, h, 36 * 1024, hipMemcpyHostToDevice, s1));
            t_h2d += us(t);
            t = Clock::now();
            CK(hipMemcpyAsync(d, h, 36 * 32768, hipMemcpyHostToDevice, s1));
            t_h2d_big += us(t);
            t = Clock::now();
            CK(hipMemcpyAsync(h, d, 8192, hipMemcpyDeviceToHost, s1));
            t_d2h += us(t);
            if ((i & 63) == 63) {
                CK(hipStreamSynchronize(s0));
                CK(hipStreamSynchronize(s1));
            }
        }
        CK(hipDeviceSynchronize());
        std::printf("rep %d per call (us): kernel 16B args %.2f, 680B args %.2f, 680B 4096 blocks %.2f, event record %.2f, "
                    "stream wait %.2f, H2D 36KB %.2f, H2D 1.2MB %.2f, D2H 8KB %.2f\n",
                    rep, t_small / N, t_big / N, t_grid / N, t_rec / N, t_wait / N, t_h2d / N, t_h2d_big / N, t_d2h / N);
    }
    return 0;
}

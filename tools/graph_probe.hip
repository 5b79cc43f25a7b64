// Launch-overhead probe: a chain of small dependent kernels plus one device->host status copy
// and a synchronisation (the shape of a C2 / C1 step's fixed cost: ~14 launches of 1 .. 4096
// workgroups, then the one read-back), run eagerly and as a replayed hipGraph.  Prints the wall
// time per chain (host clock around launch + sync) and per kernel for both.
// Usage: graph_probe [chains] [kernels per chain]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

// reads the previous kernel's word and writes its own (a real dependency, as in the pipeline)
__global__ void k_step(const unsigned* prev, unsigned* next, int i) {
    if (threadIdx.x == 0) next[blockIdx.x] = prev[blockIdx.x % 64] + (unsigned)i;
}

int main(int argc, char** argv) {
    const int chains = argc > 1 ? std::atoi(argv[1]) : 300;
    const int K = argc > 2 ? std::atoi(argv[2]) : 14;
    const unsigned grids[] = {1, 64, 512, 4096};
    unsigned *buf = nullptr, *host = nullptr;
    CK(hipMalloc(&buf, (size_t)(K + 1) * 4096 * sizeof(unsigned)));
    CK(hipMemset(buf, 0, (size_t)(K + 1) * 4096 * sizeof(unsigned)));
    CK(hipHostMalloc(&host, 4096, hipHostMallocDefault));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto enqueue = [&]() {
        for (int i = 0; i < K; ++i) {
            const unsigned grid = grids[i % 4];
            k_step<<<grid, 256, 0, s>>>(buf + (size_t)i * 4096, buf + (size_t)(i + 1) * 4096, i);
        }
        CK(hipMemcpyAsync(host, buf + (size_t)K * 4096, 1024, hipMemcpyDeviceToHost, s));
    };
    using clk = std::chrono::steady_clock;
    auto run = [&](auto&& one) {
        for (int w = 0; w < 20; ++w) { one(); CK(hipStreamSynchronize(s)); }
        std::vector<double> t(chains);
        for (int c = 0; c < chains; ++c) {
            const auto t0 = clk::now();
            one();
            CK(hipStreamSynchronize(s));
            t[c] = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
        }
        std::vector<double> u = t;
        std::sort(u.begin(), u.end());
        return std::make_pair(u[u.size() / 2], u[u.size() / 10]);
    };
    // eager
    const auto eager = run([&] { enqueue(); });
    // host enqueue cost alone (no wait inside the timed part)
    double enq = 0;
    {
        CK(hipStreamSynchronize(s));
        const auto t0 = clk::now();
        for (int c = 0; c < 50; ++c) enqueue();
        enq = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / 50;
        CK(hipStreamSynchronize(s));
    }
    // graph
    hipGraph_t graph;
    hipGraphExec_t exec;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    enqueue();
    CK(hipStreamEndCapture(s, &graph));
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    const auto gr = run([&] { CK(hipGraphLaunch(exec, s)); });
    double glaunch = 0;
    {
        CK(hipStreamSynchronize(s));
        const auto t0 = clk::now();
        for (int c = 0; c < 50; ++c) CK(hipGraphLaunch(exec, s));
        glaunch = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / 50;
        CK(hipStreamSynchronize(s));
    }
    // the kernels alone (no copy), eager: GPU-side gap per launch from events
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int c = 0; c < 100; ++c)
        for (int i = 0; i < K; ++i) k_step<<<grids[i % 4], 256, 0, s>>>(buf + (size_t)i * 4096, buf + (size_t)(i + 1) * 4096, i);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"kernels_per_chain\": %d, \"chains\": %d,\n", K, chains);
    std::printf(" \"eager_us_per_chain_median\": %.2f, \"eager_us_p10\": %.2f, \"eager_host_enqueue_us\": %.2f,\n", eager.first, eager.second, enq);
    std::printf(" \"graph_us_per_chain_median\": %.2f, \"graph_us_p10\": %.2f, \"graph_host_launch_us\": %.2f,\n", gr.first, gr.second, glaunch);
    std::printf(" \"eager_back_to_back_us_per_kernel\": %.3f}\n", ms * 1000.0 / (100.0 * K));
    std::printf("# per kernel: eager %.2f us, graph %.2f us (chain incl. the copy and the sync)\n", eager.first / K, gr.first / K);
    CK(hipGraphExecDestroy(exec));
    CK(hipGraphDestroy(graph));
    return 0;
}

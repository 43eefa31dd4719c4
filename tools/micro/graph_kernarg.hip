// HIP-graph replay probe (test infrastructure): does replaying a long-lived graph exec still
// launch its kernels with the arguments it was captured with after OTHER graph execs were instantiated, launched and
// destroyed in between?  That is the sequence under which the round-5 small-batch graph replay faulted
// (profiles/sweeps/r05_small_batch_graph_replay_tests.log: ex1000's replay after test_odd_and_small_shapes' contexts
// captured, replayed and destroyed theirs).
//
// Every buffer stays allocated until the end, so a replay that runs with another exec's arguments writes into that
// exec's (live) buffer instead of faulting: the probe counts such writes.  Each graph mimics run_batch's launch
// sequence: a memset node, then 15 kernel nodes alternating a small argument list and a ~1.5 KB by-value struct
// (OgPlan is passed by value to the octree and describe kernels).
// Mode "copies" (round 6): between two replays of one exec, the operations the round-5 fault needed on the same
// context (tests/test_gpu_extract.py::test_pyramid_and_candidates: pyramid levels read back with hipMemcpy2DAsync
// into pageable memory on the replaying stream, candidates with a synchronous hipMemcpy), each in its own round.
// Its kernels never dereference an argument they were not captured with: each checks its pointer against the buffer
// address kept in a device global and counts a mismatch there instead of writing, so corrupted arguments show as a
// count, not as a fault.
//   build: hipcc --offload-arch=gfx950 -O2 -o tools/micro/graph_kernarg tools/micro/graph_kernarg.hip
//   run:   tools/micro/graph_kernarg [rounds]           (transient execs; prints one JSON line)
//          tools/micro/graph_kernarg copies [rounds]    (copies between replays; one JSON line per operation)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                       \
        }                                                                                       \
    } while (0)

struct Big {
    long long w[190];  // 1520 bytes, like a by-value plan
};

constexpr int NK = 15, SLOTS = 64;

__device__ int* g_valid[2];   // the buffers a kernel may write (mode "copies": every other pointer is counted)
__device__ int g_bad_args;

__device__ __forceinline__ bool arg_ok(const int* p, int slot)
{
    if (!g_valid[0]) return slot >= 0 && slot < SLOTS;  // transient mode: every buffer stays allocated
    return (p == g_valid[0] || p == g_valid[1]) && slot >= 0 && slot < SLOTS;
}

__global__ void k_small(int* p, int slot, int tag)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        if (arg_ok(p, slot))
            p[slot] = tag;
        else
            atomicAdd(&g_bad_args, 1);
    }
}

__global__ void k_big(int* p, int slot, Big b)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        if (arg_ok(p, slot))
            p[slot] = (int)b.w[slot % 190];
        else
            atomicAdd(&g_bad_args, 1);
    }
}

// capture the launch sequence of one "context" writing tags base + i into buf
static hipGraphExec_t capture(hipStream_t s, int* buf, int base, void* extra = nullptr, size_t extra_bytes = 0)
{
    Big b;
    for (int i = 0; i < 190; i++) b.w[i] = base + i;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    CK(hipMemsetAsync(buf, 0, sizeof(int) * SLOTS, s));
    if (extra) CK(hipMemsetAsync(extra, 0, extra_bytes, s));
    for (int i = 0; i < NK; i++) {
        if (i & 1)
            hipLaunchKernelGGL(k_big, dim3(4), dim3(64), 0, s, buf, i, b);
        else
            hipLaunchKernelGGL(k_small, dim3(4), dim3(64), 0, s, buf, i, base + i);
    }
    hipGraph_t g = nullptr;
    CK(hipStreamEndCapture(s, &g));
    hipGraphExec_t x = nullptr;
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    return x;
}

// the tags a correct replay of `base`'s graph leaves in its buffer
static bool expected(const int* h, int base)
{
    for (int i = 0; i < NK; i++)
        if (h[i] != base + i) return false;
    for (int i = NK; i < SLOTS; i++)
        if (h[i] != 0) return false;
    return true;
}

// mode "copies": replay exec A, then one kind of operation on A's stream / the null stream, then replay A again
static int copies_mode(int rounds)
{
    hipStream_t sA;
    CK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
    int *bufA, *dev;
    CK(hipMalloc(&bufA, sizeof(int) * SLOTS));
    const int W = 640, H = 480;
    CK(hipMalloc(&dev, W * H));
    CK(hipMemset(dev, 7, W * H));
    int* valid[2] = {bufA, bufA};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_valid), valid, sizeof(valid)));
    const int zero = 0;
    std::vector<unsigned char> host(W * H);  // pageable, as a numpy array is
    std::vector<unsigned char> big_host(1 << 20);
    unsigned char *dev_big, *gbig;
    CK(hipMalloc(&dev_big, 1 << 20));
    CK(hipMemset(dev_big, 3, 1 << 20));
    CK(hipMalloc(&gbig, 1 << 16));
    std::vector<int> h(SLOTS);
    hipGraphExec_t xA = capture(sA, bufA, 1000, gbig, 1 << 16);
    const char* names[] = {"none", "memcpy2d_d2h_pitched_pageable_on_stream", "memcpy_d2h_sync_null_stream",
                           "memcpy_h2d_pageable_on_stream", "kernel_on_stream", "all_of_them",
                           "many_memcpy_d2h_sync_16KB", "many_memcpy_d2h_sync_4B", "memcpy_d2h_sync_24KB_x8",
                           "memcpy_d2h_sync_64KB_x8", "memcpy_d2h_sync_1MB_x8", "memcpy_d2h_sync_24KB_of_graph_buffer_x8"};
    int status = 0;
    for (int op = 0; op < 12; op++) {
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_bad_args), &zero, sizeof(int)));
        int bad_replays = 0;
        for (int r = 0; r < rounds; r++) {
            CK(hipGraphLaunch(xA, sA));
            CK(hipStreamSynchronize(sA));
            switch (op) {
            case 1:  // the pyramid read-back: a true 2-D region (width 533 of pitch 576, as level 1 of 640x480)
                CK(hipMemcpy2DAsync(host.data(), 533, dev, 576, 533, 400, hipMemcpyDeviceToHost, sA));
                CK(hipStreamSynchronize(sA));
                break;
            case 2:
                CK(hipMemcpy(host.data(), dev, 4096, hipMemcpyDeviceToHost));
                break;
            case 3:
                CK(hipMemcpyAsync(dev, host.data(), W * H, hipMemcpyHostToDevice, sA));
                break;
            case 4:
                hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, sA, bufA, SLOTS - 1, 0);
                break;
            case 5:  // test_pyramid_and_candidates' sequence: 8 levels, each a 2-D read-back and two synchronous copies
                for (int l = 0; l < 8; l++) {
                    CK(hipMemcpy2DAsync(host.data(), 533 - 40 * l, dev, 576, 533 - 40 * l, 400 - 30 * l,
                                        hipMemcpyDeviceToHost, sA));
                    CK(hipStreamSynchronize(sA));
                    CK(hipStreamSynchronize(sA));
                    CK(hipMemcpy(host.data(), dev, 4, hipMemcpyDeviceToHost));
                    CK(hipMemcpy(host.data(), dev, 8 * 300, hipMemcpyDeviceToHost));
                }
                break;
            case 6:  // debug_candidates at scale: synchronous D2H copies of device memory, 16 KB each
                for (int q = 0; q < 256; q++) CK(hipMemcpy(host.data(), dev, 16384, hipMemcpyDeviceToHost));
                break;
            case 7:  // ... and of 4 bytes (the per-level count)
                for (int q = 0; q < 256; q++) CK(hipMemcpy(host.data(), dev, 4, hipMemcpyDeviceToHost));
                break;
            case 8:  // the candidate read-back's sizes (8 B per candidate, thousands of candidates per level)
            case 9:
            case 10:
                for (int q = 0; q < 8; q++)
                    CK(hipMemcpy(big_host.data(), dev_big, op == 8 ? 24576 : op == 9 ? 65536 : (1 << 20),
                                 hipMemcpyDeviceToHost));
                break;
            case 11:  // a buffer the graph writes (its memset node), as the candidates are
                for (int q = 0; q < 8; q++) CK(hipMemcpy(big_host.data(), gbig, 24576, hipMemcpyDeviceToHost));
                break;
            default:
                break;
            }
            // non-zero before the replay: the graph's own memset node must clear slots NK.. (a skipped or misdirected
            // memset shows as a bad replay)
            CK(hipMemsetAsync(bufA, 0xff, sizeof(int) * SLOTS, sA));
            CK(hipGraphLaunch(xA, sA));
            CK(hipStreamSynchronize(sA));
            CK(hipMemcpy(h.data(), bufA, sizeof(int) * SLOTS, hipMemcpyDeviceToHost));
            bad_replays += !expected(h.data(), 1000);
        }
        int bad_args = 0;
        CK(hipMemcpyFromSymbol(&bad_args, HIP_SYMBOL(g_bad_args), sizeof(int)));
        const char* pc = std::getenv("DEBUG_CLR_GRAPH_PACKET_CAPTURE");
        std::printf("{\"mode\": \"copies\", \"operation\": \"%s\", \"rounds\": %d, \"bad_replays\": %d, "
                    "\"kernels_with_foreign_args\": %d, \"DEBUG_CLR_GRAPH_PACKET_CAPTURE\": \"%s\"}\n",
                    names[op], rounds, bad_replays, bad_args, pc ? pc : "(default)");
        std::fflush(stdout);
        status |= bad_replays || bad_args;
    }
    CK(hipGraphExecDestroy(xA));
    return status ? 1 : 0;
}

int main(int argc, char** argv)
{
    if (argc > 1 && std::string(argv[1]) == "copies") return copies_mode(argc > 2 ? std::atoi(argv[2]) : 16);
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 64;
    hipStream_t sA, sL;
    CK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sL, hipStreamNonBlocking));
    int *bufA, *bufL;
    CK(hipMalloc(&bufA, sizeof(int) * SLOTS));
    CK(hipMalloc(&bufL, sizeof(int) * SLOTS));
    std::vector<int*> bufT(rounds);
    for (auto& p : bufT) CK(hipMalloc(&p, sizeof(int) * SLOTS));
    // two long-lived execs (ex1000's and ex2000's), captured first
    hipGraphExec_t xA = capture(sA, bufA, 1000);
    hipGraphExec_t xL = capture(sL, bufL, 2000);
    std::vector<int> h(SLOTS);
    int bad_replays = 0, foreign_writes = 0, bad_transient = 0;
    for (int r = 0; r < rounds; r++) {
        // a transient context: own stream and graph, launched twice, then (stream synchronised) destroyed
        hipStream_t sT;
        CK(hipStreamCreateWithFlags(&sT, hipStreamNonBlocking));
        hipGraphExec_t xT = capture(sT, bufT[r], 10000 + 100 * r);
        CK(hipGraphLaunch(xT, sT));
        CK(hipGraphLaunch(xT, sT));
        CK(hipStreamSynchronize(sT));
        CK(hipMemcpy(h.data(), bufT[r], sizeof(int) * SLOTS, hipMemcpyDeviceToHost));
        bad_transient += !expected(h.data(), 10000 + 100 * r);
        CK(hipGraphExecDestroy(xT));
        CK(hipStreamDestroy(sT));
        // every transient buffer cleared, then the long-lived execs replayed
        for (int q = 0; q <= r; q++) CK(hipMemset(bufT[q], 0, sizeof(int) * SLOTS));
        CK(hipMemset(bufA, 0, sizeof(int) * SLOTS));
        CK(hipMemset(bufL, 0, sizeof(int) * SLOTS));
        CK(hipDeviceSynchronize());
        CK(hipGraphLaunch(xA, sA));
        CK(hipGraphLaunch(xL, sL));
        CK(hipStreamSynchronize(sA));
        CK(hipStreamSynchronize(sL));
        CK(hipMemcpy(h.data(), bufA, sizeof(int) * SLOTS, hipMemcpyDeviceToHost));
        bad_replays += !expected(h.data(), 1000);
        CK(hipMemcpy(h.data(), bufL, sizeof(int) * SLOTS, hipMemcpyDeviceToHost));
        bad_replays += !expected(h.data(), 2000);
        for (int q = 0; q <= r; q++) {
            CK(hipMemcpy(h.data(), bufT[q], sizeof(int) * SLOTS, hipMemcpyDeviceToHost));
            for (int i = 0; i < SLOTS; i++) foreign_writes += h[i] != 0;
        }
    }
    const char* pc = std::getenv("DEBUG_CLR_GRAPH_PACKET_CAPTURE");
    std::printf("{\"rounds\": %d, \"kernel_nodes\": %d, \"bad_long_lived_replays\": %d, \"writes_into_destroyed_execs_"
                "buffers\": %d, \"bad_transient_replays\": %d, \"DEBUG_CLR_GRAPH_PACKET_CAPTURE\": \"%s\"}\n",
                rounds, NK, bad_replays, foreign_writes, bad_transient, pc ? pc : "(default)");
    CK(hipGraphExecDestroy(xA));
    CK(hipGraphExecDestroy(xL));
    return bad_replays || foreign_writes || bad_transient ? 1 : 0;
}

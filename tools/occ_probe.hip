// Resident-wave probe: how many one-wave workgroups of a kernel run at once on
// the device, against the private-segment (scratch) and LDS bytes each wave
// holds. Every workgroup spins ~20 us and records its start and end
// (s_memrealtime); the host reports the most waves alive at once.
//
//   hipcc --offload-arch=gfx950 -O3 tools/occ_probe.hip -o tools/occ_probe && tools/occ_probe [sweep]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

template <int SCR_WORDS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void probe(unsigned long long* rec, int spin,
                                                                                     int sel) {
    extern __shared__ int lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int acc = 0;
    if constexpr (SCR_WORDS > 0) {
        volatile int buf[SCR_WORDS];                 // a private array indexed at run time: scratch
        for (int i = 0; i < SCR_WORDS; ++i) buf[i] = i ^ (int)threadIdx.x;
        acc += buf[(threadIdx.x + sel) % SCR_WORDS];
    }
    lds[threadIdx.x] = acc;
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) __builtin_amdgcn_s_sleep(2);
    acc += lds[(threadIdx.x + 1) & 63];
    if (threadIdx.x == 0) {
        rec[2 * blockIdx.x] = t0;
        rec[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() + (acc == 12345678 ? 1 : 0);
    }
}

static int peak(const std::vector<unsigned long long>& r, int n) {
    std::vector<std::pair<unsigned long long, int>> ev;
    for (int i = 0; i < n; ++i) {
        ev.push_back({r[2 * i], 1});
        ev.push_back({r[2 * i + 1], -1});
    }
    std::sort(ev.begin(), ev.end(), [](auto& a, auto& b) { return a.first < b.first || (a.first == b.first && a.second < b.second); });
    int live = 0, best = 0;
    for (auto& e : ev) best = std::max(best, live += e.second);
    return best;
}

template <int SCR>
static void run(const char* name, int lds_bytes) {
    const int n = 16384;
    unsigned long long* d;
    (void)hipMalloc(&d, sizeof(unsigned long long) * 2 * n);
    hipLaunchKernelGGL(probe<SCR>, dim3(n), dim3(64), lds_bytes, 0, d, 2000, 1);    // warm-up
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(probe<SCR>, dim3(n), dim3(64), lds_bytes, 0, d, 2000, 1);
    const hipError_t e = hipDeviceSynchronize();
    std::vector<unsigned long long> r(2 * n);
    (void)hipMemcpy(r.data(), d, sizeof(unsigned long long) * 2 * n, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    int occ = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, probe<SCR>, 64, lds_bytes);
    std::printf("{\"scratch_bytes_per_lane\": %d, \"lds_bytes\": %d, \"label\": \"%s\", \"peak_waves\": %d, "
                "\"occupancy_api_per_cu\": %d, \"err\": %d}\n",
                4 * SCR, lds_bytes, name, peak(r, n), occ, (int)e);
}

int main(int argc, char** argv) {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    std::printf("{\"cus\": %d}\n", cus);
    if (argc > 1 && std::string(argv[1]) == "sweep") {      // LDS bytes per wave against resident waves
        for (int b = 4096; b <= 12288; b += 256) run<0>("sweep", b);
        return 0;
    }
    run<0>("no scratch", 1024);
    run<0>("no scratch, comp01 LDS", 8032);
    run<0>("no scratch, comp15 LDS", 8816);
    run<0>("no scratch, compact LDS", 7552);
    run<84>("336 B scratch", 1024);
    run<84>("336 B scratch, comp01 LDS", 8032);
    run<84>("336 B scratch, compact LDS", 7552);
    run<164>("656 B scratch", 1024);
    run<32>("128 B scratch", 1024);
    return 0;
}

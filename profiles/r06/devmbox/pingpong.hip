// Development probe (round 6): round-trip latency of a one-workgroup resident
// poller, mailbox and payload in (0) mapped host memory or (1) fine-grained
// device memory written by the host, reply in mapped host memory.  Bounded:
// the kernel leaves after `iters` requests or 200 ms without one.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

__global__ void poller(const unsigned* mbox, const int4* payload, int n16, unsigned* reply, int iters) {
    __shared__ unsigned sq;
    __shared__ int sum;
    unsigned last = 0;
    for (int it = 0; it < iters; ++it) {
        if (threadIdx.x == 0) {
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            unsigned v = last;
            for (;;) {
                v = __hip_atomic_load(mbox, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (v != last) break;
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > 20000000LL) break;
                __builtin_amdgcn_s_sleep(1);
            }
            sq = v;
            sum = 0;
        }
        __syncthreads();
        const unsigned s = sq;
        if (s == last) return;
        last = s;
        int acc = 0;
        for (int i = threadIdx.x; i < n16; i += blockDim.x) {
            const int4 x = payload[i];
            acc += x.x ^ x.y ^ x.z ^ x.w;
        }
        atomicAdd(&sum, acc);
        __syncthreads();
        if (threadIdx.x == 0) {
            reply[1] = (unsigned)sum;
            __threadfence_system();
            __hip_atomic_store(reply, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static double now_us() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const int iters = 2000, n16 = 136;   // 2 176 B of payload
    unsigned* mbox;
    int4* payload;
    void* blk;
    if (mode == 0) {
        if (hipHostMalloc(&blk, 4096 + n16 * 16, hipHostMallocMapped) != hipSuccess) return 2;
    } else {
        if (hipExtMallocWithFlags(&blk, 4096 + n16 * 16, hipDeviceMallocFinegrained) != hipSuccess) return 3;
    }
    mbox = (unsigned*)blk;
    payload = (int4*)((char*)blk + 4096);
    unsigned* reply;
    if (hipHostMalloc((void**)&reply, 64, hipHostMallocMapped) != hipSuccess) return 4;
    memset((void*)reply, 0, 64);
    if (mode == 0) memset(blk, 0, 4096 + n16 * 16);
    else if (hipMemset(blk, 0, 4096 + n16 * 16) != hipSuccess) return 5;
    hipDeviceSynchronize();
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipLaunchKernelGGL(poller, dim3(1), dim3(512), 0, st, mbox, payload, n16, reply, iters);
    int4 src[136];
    for (int i = 0; i < n16; ++i) src[i] = make_int4(i, 2 * i, 3 * i, 4 * i);
    double* lat = (double*)malloc(sizeof(double) * iters);
    for (int it = 1; it <= iters; ++it) {
        const double t0 = now_us();
        src[0].x = it;
        memcpy((void*)payload, src, n16 * 16);   // host stores into the mailbox block
        if (mode) __builtin_ia32_sfence();       // (device memory: write-combined -- drain the buffers)
        __atomic_store_n(mbox, (unsigned)it, __ATOMIC_RELEASE);
        if (mode) __builtin_ia32_sfence();
        while (__atomic_load_n(reply, __ATOMIC_ACQUIRE) != (unsigned)it) {
            if (now_us() - t0 > 100000) { fprintf(stderr, "timeout at %d\n", it); hipStreamSynchronize(st); return 6; }
        }
        lat[it - 1] = now_us() - t0;
    }
    hipStreamSynchronize(st);
    // median
    for (int i = 0; i < iters; ++i)
        for (int j = i + 1; j < iters; ++j)
            if (lat[j] < lat[i]) { double x = lat[i]; lat[i] = lat[j]; lat[j] = x; }
    printf("mode %d (%s): median %.2f us, p10 %.2f, p90 %.2f\n", mode, mode ? "device fine-grained" : "mapped host",
           lat[iters / 2], lat[iters / 10], lat[iters * 9 / 10]);
    return 0;
}

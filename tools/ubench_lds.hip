// Microbenchmark: LDS float atomic throughput vs plain LDS read-modify-write on gfx950.
// Used to decide the splat design (DESIGN.md "Splat"). Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 4096;
constexpr int kLds = 8192;

template <int MODE>
__global__ __launch_bounds__(1024) void k(float* out, int stride) {
    __shared__ float s[kLds];
    for (int i = threadIdx.x; i < kLds; i += blockDim.x) s[i] = 0.f;
    __syncthreads();
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float v = 1.0f + lane * 1e-3f;
    for (int it = 0; it < kIters; ++it) {
        int a;
        if (MODE == 2) a = (w * 97 + it * 7) & (kLds - 1);                   // whole wave same address
        else a = (w * 512 + lane * stride + it * 5) & (kLds - 1);             // distinct per lane
        if (MODE == 0 || MODE == 2) atomicAdd(&s[a], v);
        else if (MODE == 1) { s[a] += v; }                                    // plain RMW (racy, timing only)
        else if (MODE == 3) __hip_atomic_fetch_add(&s[a], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else if (MODE == 4) atomicAdd((unsigned*)&s[a], (unsigned)(lane + 1));
        else if (MODE == 5) atomicAdd((unsigned long long*)&s[a & ~1], (unsigned long long)(lane + 1));
        else if (MODE == 6) { float r = atomicAdd(&s[a], v); v += r * 1e-30f; }
        else if (MODE == 7) unsafeAtomicAdd(&out[1 + ((blockIdx.x * 4096 + (threadIdx.x + it * 64) ) & ((1 << 20) - 1))], v);
        else if (MODE == 9) {
            unsigned* p = (unsigned*)&s[a];
            unsigned old = *p;
            while (true) {
                unsigned nw = __float_as_uint(__uint_as_float(old) + v);
                unsigned prev = __hip_atomic_compare_exchange_strong(p, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ? old : old;
                if (prev == old && __float_as_uint(__uint_as_float(old) + v) == nw) break;
            }
        }
        else if (MODE == 10) {
            unsigned* p = (unsigned*)&s[(w * 97 + it * 7 + (lane & 3)) & (kLds - 1)];
            unsigned old = *p;
            while (!__hip_atomic_compare_exchange_strong(p, &old, __float_as_uint(__uint_as_float(old) + v), __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {}
        }
        else if (MODE == 11) atomicAdd((double*)&s[a & ~1], (double)v);
        else if (MODE == 12) {   /* fixed-point (32 fractional bits) f32 -> u64, ds_add_u64 */
            const float x = v * 4294967296.f;
            const unsigned hi = (unsigned)(x * 2.3283064365386963e-10f);
            const unsigned lo = (unsigned)__builtin_fmaf(-(float)hi, 4294967296.f, x);
            atomicAdd((unsigned long long*)&s[a & ~1], ((unsigned long long)hi << 32) + lo);
        }
        else if (MODE == 13) {   /* 64-bit CAS of a float pair (the current splat window) */
            unsigned long long* p = (unsigned long long*)&s[a & ~1];
            unsigned long long old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            while (true) {
                unsigned long long nw = (unsigned long long)__float_as_uint(__uint_as_float((unsigned)old) + v) |
                                        ((unsigned long long)__float_as_uint(__uint_as_float((unsigned)(old >> 32)) + v) << 32);
                if (__hip_atomic_compare_exchange_strong(p, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
            }
        }
        else if (MODE == 14) atomicAdd((unsigned long long*)&s[(a * 2) & (kLds - 2)], (unsigned long long)(lane + 1));
        else if (MODE == 15) atomicAdd((double*)&s[(a * 2) & (kLds - 2)], (double)v);
        else if (MODE == 16) {
            const float x = v * 4294967296.f;
            const unsigned hi = (unsigned)(x * 2.3283064365386963e-10f);
            const unsigned lo = (unsigned)__builtin_fmaf(-(float)hi, 4294967296.f, x);
            atomicAdd((unsigned long long*)&s[(a * 2) & (kLds - 2)], ((unsigned long long)hi << 32) + lo);
        }
        else if (MODE == 8) { float x = s[a]; __builtin_amdgcn_s_waitcnt(0); s[a] = x + v; }
    }
    __syncthreads();
    float acc = 0.f;
    for (int i = threadIdx.x; i < kLds; i += blockDim.x) acc += s[i];
    if (acc == 12345.f) out[0] = acc;
}

template <int MODE>
void run(const char* name, int stride, int block) {
    float* d; (void)hipMalloc(&d, 8 << 20);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    int grid = 256 * 8;
    k<MODE><<<grid, block>>>(d, stride);
    hipEventRecord(a);
    k<MODE><<<grid, block>>>(d, stride);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double ops = double(grid) * block * kIters;
    printf("%-34s stride %2d block %4d: %8.3f ms  %8.1f Glane-ops/s  %6.2f lane-ops/clk/CU\n", name, stride, block, ms,
           ops / ms / 1e6, ops / (ms * 1e-3) / 256 / 2.4e9);
    hipFree(d);
}

int main() {
    for (int bs : {512}) {
        run<5>("ds_add_u64 distinct", 1, bs);
        run<14>("ds_add_u64 distinct 8B-stride", 1, bs);
        run<11>("ds_add_f64 distinct", 1, bs);
        run<15>("ds_add_f64 distinct 8B-stride", 1, bs);
        run<16>("fixed-point cvt + u64 8B-stride", 1, bs);
        run<12>("fixed-point cvt + ds_add_u64", 1, bs);
        run<13>("CAS64 pair add distinct", 1, bs);
        run<4>("ds_add_u32 distinct", 1, bs);
        run<9>("CAS-loop f32 add distinct", 1, bs);
    }
    for (int bs : {256, 1024}) {
        run<0>("ds_add_f32 distinct", 1, bs);
        run<0>("ds_add_f32 distinct", 3, bs);
        run<0>("ds_add_f32 distinct", 32, bs);
        run<2>("ds_add_f32 same-address", 0, bs);
        run<1>("ds_read+ds_write", 1, bs);
        run<3>("fetch_add workgroup", 1, bs);
        run<4>("ds_add_u32 distinct", 1, bs);
        run<5>("ds_add_u64 distinct", 2, bs);
        run<6>("ds_add_rtn_f32 distinct", 1, bs);
        run<7>("global unsafeAtomicAdd 4MB", 1, bs);
        run<8>("ds_read;wait;ds_write", 1, bs);
        run<9>("CAS-loop f32 add distinct", 1, bs);
        run<10>("CAS-loop f32 add 16-way contention", 1, bs);
    }
    return 0;
}

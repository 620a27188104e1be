// d16_probe.hip -- does ds_read_u16_d16_hi keep the low half of its VGPR on
// this GPU?  LLVM only emits the preserving d16 LDS loads for sramecc-
// targets; this checks the hardware behaviour before the pixel kernel relies
// on it (tools/microbench, tuning only).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void probe(uint32_t* out)
{
    __shared__ unsigned short lds[256];
    const int t = threadIdx.x;
    lds[t] = static_cast<unsigned short>(0x1000 + t);
    lds[128 + t] = static_cast<unsigned short>(0xA000 + t);
    __syncthreads();
    uint32_t v = 0x5555u + static_cast<uint32_t>(t);   // low half must survive
    // LDS byte addresses derived from the array (keeps its stores alive)
    const uint32_t base = static_cast<uint32_t>(reinterpret_cast<size_t>(lds));
    const uint32_t addr = base + static_cast<uint32_t>((128 + t) * 2);
    asm volatile("ds_read_u16_d16_hi %0, %1\n s_waitcnt lgkmcnt(0)" : "+v"(v) : "v"(addr) : "memory");
    uint32_t w = 0;
    const uint32_t addr2 = base + static_cast<uint32_t>(t * 2);
    asm volatile("ds_read_u16 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(addr2) : "memory");
    asm volatile("ds_read_u16_d16_hi %0, %1\n s_waitcnt lgkmcnt(0)" : "+v"(w) : "v"(addr) : "memory");
    out[2 * t] = v;
    out[2 * t + 1] = w;
}

int main()
{
    uint32_t* d;
    if (hipMalloc(&d, 1024) != hipSuccess) return 2;
    probe<<<1, 64>>>(d);
    uint32_t h[128];
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
    int bad = 0;
    for (int t = 0; t < 64; ++t) {
        const uint32_t e1 = ((0xA000u + t) << 16) | (0x5555u + t);
        const uint32_t e2 = ((0xA000u + t) << 16) | (0x1000u + t);
        if (h[2 * t] != e1 || h[2 * t + 1] != e2) {
            if (bad < 4) printf("lane %d: %08x (want %08x)  %08x (want %08x)\n", t, h[2 * t], e1, h[2 * t + 1], e2);
            ++bad;
        }
    }
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 4;
    printf("arch %s: ds_read_u16_d16_hi preserves the low half: %s (%d bad lanes)\n", p.gcnArchName, bad ? "NO" : "yes", bad);
    return bad ? 1 : 0;
}

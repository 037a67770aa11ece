#include <hip/hip_runtime.h>
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2(float2v x, half2v &hi, half2v &lo) {
    hi = __builtin_convertvector(x, half2v);
    unsigned h = __builtin_bit_cast(unsigned, hi), l = 0;
    asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %0, -%1, 1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "+v"(l) : "v"(h), "v"(x.x), "v"(x.y));
    lo = __builtin_bit_cast(half2v, l);
}
__global__ void k(half2v *oh, half2v *ol, const float2v *x) {
    int l = threadIdx.x;
    half2v hi, lo;
    split2(x[l], hi, lo);
    oh[l] = hi; ol[l] = lo;
}
int main() {
    const int N = 64;
    float2v hx[N]; half2v hh[N], hl[N];
    for (int i = 0; i < N; ++i) { hx[i].x = 1.0f / (i + 3) * (i % 2 ? -1 : 1) * 1000.f; hx[i].y = 0.1234567f * i - 3.3f; }
    float2v *dx; half2v *dh, *dl;
    hipMalloc(&dx, sizeof(hx)); hipMalloc(&dh, sizeof(hh)); hipMalloc(&dl, sizeof(hl));
    hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice);
    k<<<1, N>>>(dh, dl, dx);
    hipMemcpy(hh, dh, sizeof(hh), hipMemcpyDeviceToHost); hipMemcpy(hl, dl, sizeof(hl), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < N; ++i) {
        for (int c = 0; c < 2; ++c) {
            float x = c ? hx[i].y : hx[i].x;
            _Float16 h = (_Float16)x, lref = (_Float16)(x - (float)h);
            _Float16 hg = c ? hh[i].y : hh[i].x, lg = c ? hl[i].y : hl[i].x;
            if (__builtin_bit_cast(unsigned short, hg) != __builtin_bit_cast(unsigned short, h) ||
                __builtin_bit_cast(unsigned short, lg) != __builtin_bit_cast(unsigned short, lref)) {
                if (bad < 5) printf("mismatch i=%d c=%d x=%g lo %g vs %g\n", i, c, x, (float)lg, (float)lref);
                ++bad;
            }
        }
    }
    printf("split2 fma_mix check: %d mismatches of %d\n", bad, 2 * N);
    return bad != 0;
}

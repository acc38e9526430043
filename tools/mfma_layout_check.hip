// mfma_layout_check.hip — verifies the operand/result lane maps of the i8 and
// f32-input MFMAs used by the prefill kernel, with exact integer data and an
// asymmetric B (guide: "check the map with exact integer data").
//   assumed maps (32x32x32 i8): lane l, r = l&31, h = l>>5:
//     A[row r][k = 16h + j], B[k = 16h + j][col r], j = 0..15 (bytes of 4 VGPRs)
//     C/D: col = l&31, row = (reg&3) + 8*(reg>>2) + 4*h, reg = 0..15
//   32x32x2 f32: A[r][k = h], B[k = h][col r]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k_i8(const signed char *A, const signed char *B, int *C) {  // A 32x32 row-major [m][k], B [k][n]
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    i32x4 a, b;
    signed char *pa = (signed char *)&a, *pb = (signed char *)&b;
    for (int j = 0; j < 16; ++j) {
        pa[j] = A[r * 32 + 16 * h + j];
        pb[j] = B[(16 * h + j) * 32 + r];
    }
    i32x16 c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    for (int reg = 0; reg < 16; ++reg) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h, col = r;
        C[row * 32 + col] = c[reg];
    }
}

__global__ void k_f32(const float *A, const float *B, float *C) {  // A 32x2 [m][k], B 2x32 [k][n]
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    f32x16 c = {};
    c = __builtin_amdgcn_mfma_f32_32x32x2f32(A[r * 2 + h], B[h * 32 + r], c, 0, 0, 0);
    for (int reg = 0; reg < 16; ++reg) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h, col = r;
        C[row * 32 + col] = c[reg];
    }
}

int main() {
    signed char hA[1024], hB[1024];
    int hC[1024], ref[1024];
    srand(7);
    for (int i = 0; i < 1024; ++i) {
        hA[i] = (signed char)(rand() % 255 - 127);
        hB[i] = (signed char)(rand() % 255 - 127);
    }
    for (int m = 0; m < 32; ++m)
        for (int n = 0; n < 32; ++n) {
            int s = 0;
            for (int k = 0; k < 32; ++k) s += hA[m * 32 + k] * hB[k * 32 + n];
            ref[m * 32 + n] = s;
        }
    signed char *dA, *dB;
    int *dC;
    hipMalloc(&dA, 1024);
    hipMalloc(&dB, 1024);
    hipMalloc(&dC, 4096);
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_i8, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 1024; ++i) bad += hC[i] != ref[i];
    printf("i8 32x32x32 map: %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);

    float fA[64], fB[64], fC[1024], fref[1024];
    for (int i = 0; i < 64; ++i) {
        fA[i] = (float)(rand() % 2001 - 1000);
        fB[i] = (float)(rand() % 2001 - 1000);
    }
    for (int m = 0; m < 32; ++m)
        for (int n = 0; n < 32; ++n) fref[m * 32 + n] = fA[m * 2] * fB[n] + fA[m * 2 + 1] * fB[32 + n];
    float *dfA, *dfB, *dfC;
    hipMalloc(&dfA, 256);
    hipMalloc(&dfB, 256);
    hipMalloc(&dfC, 4096);
    hipMemcpy(dfA, fA, 256, hipMemcpyHostToDevice);
    hipMemcpy(dfB, fB, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_f32, dim3(1), dim3(64), 0, 0, dfA, dfB, dfC);
    hipMemcpy(fC, dfC, 4096, hipMemcpyDeviceToHost);
    bad = 0;
    for (int i = 0; i < 1024; ++i) bad += fC[i] != fref[i];
    printf("f32 32x32x2 map: %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
    return 0;
}

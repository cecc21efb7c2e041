// Probe (diagnostic): operand/result lane maps of v_mfma_i32_16x16x64_i8 on gfx950.
// Each lane passes 16 i8 of A and 16 i8 of B (4 VGPRs each) and gets 4 i32 of C.
// The host checks candidate maps against a CPU product of the same bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const int8_t *A, const int8_t *B, int *C)
{
    const int l = threadIdx.x;
    v4i a, b;
    __builtin_memcpy(&a, A + 16 * l, 16);
    __builtin_memcpy(&b, B + 16 * l, 16);
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; r++)
        C[4 * l + r] = c[r];
}
int main()
{
    int8_t hA[1024], hB[1024];
    srand(7);
    for (int i = 0; i < 1024; i++) {
        hA[i] = (int8_t)(rand() % 255 - 127);
        hB[i] = (int8_t)(rand() % 255 - 127);
    }
    int8_t *dA, *dB;
    int *dC, hC[256];
    hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 1024);
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
    // candidate k maps for (lane-group g = l >> 4, byte j): k = 16 g + j  |  8 g + j (+32 for j >= 8)
    for (int cand = 0; cand < 2; cand++) {
        int bad = 0;
        for (int l = 0; l < 64; l++)
            for (int r = 0; r < 4; r++) {
                const int row = 4 * (l >> 4) + r, col = l & 15;  // C map: col = lane & 15, row = 4 (lane >> 4) + r
                long s = 0;
                for (int L = 0; L < 64; L++) {  // lanes holding A row `row` and B col `col`
                    for (int j = 0; j < 16; j++) {
                        // A element of lane L byte j is A[L & 15][k(L>>4, j)]; B likewise B[k][L & 15]
                        (void)L; (void)j;
                    }
                }
                // direct: C[row][col] = sum_k A[row][k] B[k][col]
                for (int kk = 0; kk < 64; kk++) {
                    int g, j;
                    if (cand == 0) { g = kk / 16; j = kk % 16; }
                    else { g = (kk % 32) / 8; j = (kk % 8) + 8 * (kk / 32); }
                    s += (long)hA[16 * (16 * g + row) + j] * hB[16 * (16 * g + col) + j];
                }
                if (s != hC[4 * l + r])
                    bad++;
            }
        printf("candidate %d: %d mismatches of 256\n", cand, bad);
    }
    return 0;
}

// mfma_hazard.hip -- wait states needed around v_mfma_f32_16x16x32_f16 on gfx950
// (diagnostic tool, not product code).  Every wave runs a hand-placed sequence with
// K s_nop wait states between an MFMA and a dependent instruction, on exactly
// representable data, and counts wrong results:
//   raw : MFMA writes v[40:43]; K nops; VALU reads v40
//   war : MFMA reads C = v[40:43] (writes v[44:47]); K nops; VALU overwrites v40;
//         long wait; VALU reads v44 (wrong if the MFMA read the overwritten C)
//   srcc: MFMA writes v[40:43]; K nops; a second MFMA reads it as C (different D)
// 16 waves per CU x every CU, many repetitions, so the XDL pipes are contended.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_hazard_bin tools/mfma_hazard.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));


template <int K>
__global__ void __launch_bounds__(1024) k_raw(unsigned* bad, int reps) {
  half8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)(1 + (threadIdx.x + j) % 3); b[j] = (_Float16)(1 + j % 2); }
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], %1, %2, 0\n"
        "s_nop %3\n"
        "v_mov_b32 %0, v40\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n"
        : "=v"(v) : "v"(a), "v"(b), "n"(K) : "v40", "v41", "v42", "v43");
    nbad += (v == 0.f) ? 1u : 0u;  // every product is >= 1: 0 = read before written
  }
  if (nbad) atomicAdd(bad, nbad);
}

template <int K>
__global__ void __launch_bounds__(1024) k_war(unsigned* bad, int reps) {
  half8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)1; b[j] = (_Float16)1; }
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v40, 1000.0\n v_mov_b32 v41, 1000.0\n v_mov_b32 v42, 1000.0\n v_mov_b32 v43, 1000.0\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[44:47], %1, %2, v[40:43]\n"
        "s_nop %3\n"
        "v_mov_b32 v40, 0\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
        "v_mov_b32 %0, v44\n"
        : "=v"(v) : "v"(a), "v"(b), "n"(K) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
    nbad += (v != 1032.f) ? 1u : 0u;  // 32 ones + C = 1000
  }
  if (nbad) atomicAdd(bad, nbad);
}

template <int K>
__global__ void __launch_bounds__(1024) k_srcc(unsigned* bad, int reps) {
  half8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)1; b[j] = (_Float16)1; }
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], %1, %2, 0\n"
        "s_nop %3\n"
        "v_mfma_f32_16x16x32_f16 v[44:47], %1, %2, v[40:43]\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
        "v_mov_b32 %0, v44\n"
        : "=v"(v) : "v"(a), "v"(b), "n"(K) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
    nbad += (v != 64.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// MFMA writes v[40:43]; K nops; a packed 64-bit VALU (v_pk_add_f32) reads v[40:41]
template <int K>
__global__ void __launch_bounds__(1024) k_rawpk(unsigned* bad, int reps) {
  half8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)1; b[j] = (_Float16)1; }
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n v_mov_b32 v48, 0\n v_mov_b32 v49, 0\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], %1, %2, 0\n"
        "s_nop %3\n"
        "v_pk_add_f32 v[48:49], v[40:41], v[48:49]\n"
        "s_nop 7\n s_nop 7\n"
        "v_mov_b32 %0, v49\n"
        : "=v"(v) : "v"(a), "v"(b), "n"(K) : "v40", "v41", "v42", "v43", "v48", "v49");
    nbad += (v != 32.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// MFMA writes v[40:43]; K nops; v_pk_mul_f32 with an SGPR pair reads v[42:43] (as hipcc emits)
template <int K>
__global__ void __launch_bounds__(1024) k_rawpks(unsigned* bad, int reps) {
  half8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)1; b[j] = (_Float16)1; }
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n"
        "s_mov_b32 s60, 1.0\n s_mov_b32 s61, 1.0\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], %1, %2, 0\n"
        "s_nop %3\n"
        "v_pk_mul_f32 v[48:49], v[42:43], s[60:61] op_sel_hi:[1,0]\n"
        "s_nop 7\n s_nop 7\n"
        "v_mov_b32 %0, v49\n"
        : "=v"(v) : "v"(a), "v"(b), "n"(K) : "v40", "v41", "v42", "v43", "v48", "v49", "s60", "s61");
    nbad += (v != 32.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// MFMA writes v[40:43]; K nops; VALU reads the LAST result register v43 (v_mov) / v[42:43] (v_pk_add)
template <int K>
__global__ void __launch_bounds__(1024) k_raw43(unsigned* bad, int reps) {
  half8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)1; b[j] = (_Float16)1; }
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], %1, %2, 0\n"
        "s_nop %3\n"
        "v_mov_b32 %0, v43\n"
        "s_nop 7\n s_nop 7\n"
        : "=v"(v) : "v"(a), "v"(b), "n"(K) : "v40", "v41", "v42", "v43");
    nbad += (v != 32.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}
template <int K>
__global__ void __launch_bounds__(1024) k_rawpk43(unsigned* bad, int reps) {
  half8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)1; b[j] = (_Float16)1; }
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n v_mov_b32 v48, 0\n v_mov_b32 v49, 0\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], %1, %2, 0\n"
        "s_nop %3\n"
        "v_pk_add_f32 v[48:49], v[42:43], v[48:49]\n"
        "s_nop 7\n s_nop 7\n"
        "v_mov_b32 %0, v49\n"
        : "=v"(v) : "v"(a), "v"(b), "n"(K) : "v40", "v41", "v42", "v43", "v48", "v49");
    nbad += (v != 32.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// f32-input MFMA (v_mfma_f32_16x16x4_f32, the round-1 kernels): last result register
template <int K>
__global__ void __launch_bounds__(1024) k_raw43f32(unsigned* bad, int reps) {
  const float a = 1.f, b = 1.f;
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x4_f32 v[40:43], %1, %2, 0\n"
        "s_nop %3\n"
        "v_mov_b32 %0, v43\n"
        "s_nop 7\n s_nop 7\n"
        : "=v"(v) : "v"(a), "v"(b), "n"(K) : "v40", "v41", "v42", "v43");
    nbad += (v != 4.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// v_cvt_pkrtz_f16_f32 writes the B operand (v[52:55], as split8 does); K nops; MFMA reads it
template <int K>
__global__ void __launch_bounds__(1024) k_cvt2b(unsigned* bad, int reps) {
  half8 a;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = (_Float16)1;
  unsigned nbad = 0;
  const float one = 1.0f + 0.0f * threadIdx.x;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n v_mov_b32 v54, 0\n v_mov_b32 v55, 0\n"
        "s_nop 7\n s_nop 7\n"
        "v_cvt_pkrtz_f16_f32 v52, %2, %2\n v_cvt_pkrtz_f16_f32 v53, %2, %2\n"
        "v_cvt_pkrtz_f16_f32 v54, %2, %2\n v_cvt_pkrtz_f16_f32 v55, %2, %2\n"
        "s_nop %3\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], %1, v[52:55], 0\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n"
        "v_mov_b32 %0, v40\n"
        : "=v"(v) : "v"(a), "v"(one), "n"(K) : "v40", "v41", "v42", "v43", "v52", "v53", "v54", "v55");
    nbad += (v != 32.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// v_perm_b32 writes the B operand; K nops; MFMA reads it
template <int K>
__global__ void __launch_bounds__(1024) k_perm2b(unsigned* bad, int reps) {
  half8 a;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = (_Float16)1;
  unsigned nbad = 0;
  const unsigned one = 0x3c003c00u + 0u * threadIdx.x;
  const unsigned sel = 0x05040100u + 0u * threadIdx.x;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n v_mov_b32 v54, 0\n v_mov_b32 v55, 0\n"
        "s_nop 7\n s_nop 7\n"
        "v_perm_b32 v52, %2, %2, %4\n v_perm_b32 v53, %2, %2, %4\n"
        "v_perm_b32 v54, %2, %2, %4\n v_perm_b32 v55, %2, %2, %4\n"
        "s_nop %3\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], %1, v[52:55], 0\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n"
        "v_mov_b32 %0, v40\n"
        : "=v"(v) : "v"(a), "v"(one), "n"(K), "v"(sel) : "v40", "v41", "v42", "v43", "v52", "v53", "v54", "v55");
    nbad += (v != 32.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// MFMA reads A = v[48:51]; K nops; a VALU overwrites the LAST A register (WAR on SrcA)
template <int K>
__global__ void __launch_bounds__(1024) k_wara(unsigned* bad, int reps) {
  half8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (_Float16)1;
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v48, 0x3c003c00\n v_mov_b32 v49, 0x3c003c00\n v_mov_b32 v50, 0x3c003c00\n v_mov_b32 v51, 0x3c003c00\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], v[48:51], %1, 0\n"
        "s_nop %2\n"
        "v_mov_b32 v51, 0\n v_mov_b32 v50, 0\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n"
        "v_mov_b32 %0, v40\n"
        : "=v"(v) : "v"(b), "n"(K) : "v40", "v41", "v42", "v43", "v48", "v49", "v50", "v51");
    nbad += (v != 32.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// MFMA reads B = v[52:55]; K nops; a VALU overwrites the last B register (WAR on SrcB)
template <int K>
__global__ void __launch_bounds__(1024) k_warb(unsigned* bad, int reps) {
  half8 a;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = (_Float16)1;
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v52, 0x3c003c00\n v_mov_b32 v53, 0x3c003c00\n v_mov_b32 v54, 0x3c003c00\n v_mov_b32 v55, 0x3c003c00\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], %1, v[52:55], 0\n"
        "s_nop %2\n"
        "v_mov_b32 v55, 0\n v_mov_b32 v54, 0\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n"
        "v_mov_b32 %0, v40\n"
        : "=v"(v) : "v"(a), "n"(K) : "v40", "v41", "v42", "v43", "v52", "v53", "v54", "v55");
    nbad += (v != 32.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// MFMA result (last register) stored by a global store after K nops
template <int K>
__global__ void __launch_bounds__(1024) k_raw2store(unsigned* bad, float* sink, int reps) {
  half8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)1; b[j] = (_Float16)1; }
  float* dst = sink + (blockIdx.x * blockDim.x + threadIdx.x);
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    asm volatile(
        "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], %0, %1, 0\n"
        "s_nop %3\n"
        "global_store_dword %2, v43, off\n"
        "s_waitcnt vmcnt(0)\n"
        : : "v"(a), "v"(b), "v"(dst), "n"(K) : "v40", "v41", "v42", "v43", "memory");
    nbad += (*(volatile float*)dst != 32.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// VALU writes the A operand (v[48:51]); K nops; MFMA reads it
template <int K>
__global__ void __launch_bounds__(1024) k_valu2a(unsigned* bad, int reps) {
  half8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (_Float16)1;
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v48, 0\n v_mov_b32 v49, 0\n v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n"
        "s_nop 7\n s_nop 7\n"
        "v_mov_b32 v48, 0x3c003c00\n v_mov_b32 v49, 0x3c003c00\n v_mov_b32 v50, 0x3c003c00\n v_mov_b32 v51, 0x3c003c00\n"
        "s_nop %2\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], v[48:51], %1, 0\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n"
        "v_mov_b32 %0, v40\n"
        : "=v"(v) : "v"(b), "n"(K) : "v40", "v41", "v42", "v43", "v48", "v49", "v50", "v51");
    nbad += (v != 32.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

// D overlaps A (v_mfma v[40:43], v[40:43], B, 0), then the result is read after 7 states
template <int K>
__global__ void __launch_bounds__(1024) k_dsta(unsigned* bad, int reps) {
  half8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = (_Float16)1;
  unsigned nbad = 0;
  for (int r = 0; r < reps; ++r) {
    float v;
    asm volatile(
        "v_mov_b32 v40, 0x3c003c00\n v_mov_b32 v41, 0x3c003c00\n v_mov_b32 v42, 0x3c003c00\n v_mov_b32 v43, 0x3c003c00\n"
        "s_nop 7\n s_nop 7\n"
        "v_mfma_f32_16x16x32_f16 v[40:43], v[40:43], %1, 0\n"
        "s_nop %2\n"
        "s_nop 7\n s_nop 7\n s_nop 7\n"
        "v_mov_b32 %0, v40\n"
        : "=v"(v) : "v"(b), "n"(K) : "v40", "v41", "v42", "v43");
    nbad += (v != 32.f) ? 1u : 0u;
  }
  if (nbad) atomicAdd(bad, nbad);
}

static unsigned run(void (*k)(unsigned*, int), unsigned* d) {
  hipMemset(d, 0, 4);
  hipLaunchKernelGGL(k, dim3(1024), dim3(1024), 0, 0, d, 200);
  unsigned h = 0;
  hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  return h;
}

#define ROW(name, K) printf("%-5s K=%2d  wrong %u of %u\n", #name, K, run(k_##name<K>, d), 1024u * 1024u * 200u)

static unsigned run_s(void (*k)(unsigned*, float*, int), unsigned* d, float* sink) {
  hipMemset(d, 0, 4);
  hipLaunchKernelGGL(k, dim3(1024), dim3(1024), 0, 0, d, sink, 200);
  unsigned h = 0;
  hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  return h;
}
#define ROWS(name, K) printf("%-8s K=%2d  wrong %u of %u\n", #name, K, run_s(k_##name<K>, d, sink), 1024u * 1024u * 200u)

int main() {
  unsigned* d;
  hipMalloc(&d, 4);
  float* sink;
  hipMalloc(&sink, 1024 * 1024 * 4);
  ROW(wara, 0); ROW(wara, 1); ROW(wara, 2); ROW(wara, 3);
  ROW(warb, 0); ROW(warb, 1); ROW(warb, 2); ROW(warb, 3);
  return 0;
}

// Per-launch time of one mlp_phase_kernel job (csrc/mlp_kernels.hip) in a
// graph chain of R identical launches: C[M][N] = act(A[M][K] B[N][K]^T + b).
// usage: mlp_phase_micro M N K RI RJ mode(depth | 100 lds) [R]
#include "../h2omx/csrc/mlp_kernels.hip"
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  if (argc < 7) { printf("usage\n"); return 1; }
  const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]), RI = atoi(argv[4]), RJ = atoi(argv[5]);
  const int mode = atoi(argv[6]), R = argc > 7 ? atoi(argv[7]) : 50;
  float *A, *B, *C, *bias;
  CK(hipMalloc(&A, (size_t)M * K * 4)); CK(hipMalloc(&B, (size_t)N * K * 4));
  CK(hipMalloc(&C, (size_t)M * N * 4)); CK(hipMalloc(&bias, (size_t)N * 4));
  std::vector<float> h((size_t)std::max(M, N) * K);
  for (auto& v : h) v = (rand() % 1000) * 1e-3f - 0.5f;
  CK(hipMemcpy(A, h.data(), (size_t)M * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), (size_t)N * K * 4, hipMemcpyHostToDevice));
  CK(hipMemset(bias, 0, N * 4));
  Phase ph{};
  ph.ng = 1; ph.na = 0; ph.pad = mode;
  GemmJob& j = ph.g[0];
  j.A = Opnd{A, K, 1, 1}; j.B = Opnd{B, K, 1, 1};  // both K-contiguous, aligned
  j.I = M; j.J = N; j.K = K; j.RI = RI; j.RJ = RJ;
  j.tiles_j = (N + 16 * RJ - 1) / (16 * RJ);
  j.tiles = j.tiles_j * ((M + 16 * RI - 1) / (16 * RI));
  j.epi = 0; j.act = 1; j.out = C; j.ldo = N; j.bias = bias;
  hipStream_t s; CK(hipStreamCreate(&s));
  for (int w = 0; w < 3; ++w) if (h2omx_mlp_phase(&ph, s) != 0) { printf("launch failed\n"); return 1; }
  CK(hipStreamSynchronize(s));
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int r = 0; r < R; ++r) h2omx_mlp_phase(&ph, s);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int it = 0; it < 5; ++it) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("M=%d N=%d K=%d RI=%d RJ=%d mode=%d tiles=%d: %.2f us/launch (%.1f TFLOP/s)\n", M, N, K, RI, RJ, mode,
         j.tiles, 1000.f * ms / (5 * R), 2.0 * M * N * K / (1e-3 * ms / (5 * R)) / 1e12);
  return 0;
}

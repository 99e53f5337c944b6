// Diagnostic build of the fused intra kernel with phase ablation (tools/ablate/run.py).
// Not part of libivc: compiled separately with IVC_ABLATION; outputs are meaningless when a
// phase is skipped, only the timing is read.  ng selects the load-tile width (1, 2, 4, 8).
#define IVC_ABLATION 1
#include "../../ivclab_amd/csrc/ivc_kernels.hip"

extern "C" int diag_intra_u8(const void* img, int64_t F, int64_t H, int64_t W,
                             const double* table, int32_t* out, int ablate, int ng, int reps,
                             float* ms) {
  using namespace ivc;
  QTab t;
  for (int i = 0; i < 192; ++i) t.q[i] = table[i];
  FusedArgs a = make_fused_args(img, nullptr, out, F, H, W, 0, t);
  a.ablate = ablate;
  auto launch = [&]() {
    switch (ng) {
      case 1: launch_fused_one<uint8_t, double, double, 1, true, false, SRC_IMAGE, false, 1>(a, t, 0); break;
      case 2: launch_fused_one<uint8_t, double, double, 1, true, false, SRC_IMAGE, false, 2>(a, t, 0); break;
      case 8: launch_fused_one<uint8_t, double, double, 1, true, false, SRC_IMAGE, false, 8>(a, t, 0); break;
      default: launch_fused_one<uint8_t, double, double, 1, true, false, SRC_IMAGE, false, 4>(a, t, 0); break;
    }
  };
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch();
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(ms, e0, e1);
  *ms /= reps;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return (int)hipGetLastError();
}

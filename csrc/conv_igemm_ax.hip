// Instantiations of the implicit-GEMM kernel (conv_nt_kernel.h) with the BatchNorm apply
// folded into the A-operand staging (AXArgs): mode 1 = the forward bn3(+residual)+ReLU
// of the previous ResNet block applied by the next block's conv1 (plain epilogue, BN
// statistics of conv1's output); mode 2 = the bn3 backward apply applied by conv3's
// data-gradient GEMM (with the fused bn2 BatchNorm-backward epilogue); mode 3 = bn2's
// backward apply (ReLU gate recomputed from y2) in conv2's 3x3 data gradient (with bn1's).
// Register-staged tiles apply it while staging; LDS-DMA tiles (20..28; not 21, whose BN-backward
// instantiation spills) rewrite the landed A tile in LDS.
// A separate translation unit like conv_igemm_bnb.hip.
#include "conv_nt_kernel.h"

namespace pdt_nt {

// the 256x64 register-staged tiles (1, 6, 16) spill 2 VGPRs in mode 3: mode 3 returns
// NOT_APPLICABLE for them (their case labels name the mode-2 kernel only so that no mode-3
// instantiation is emitted; it is never launched)
template <int AX, bool BNB>
static int launch_ax(int v, const NTParams& p, hipStream_t st) {
  if constexpr (AX == 3) {
    if (v == 1 || v == 6 || v == 16) return -5;
  }
  switch (v) {
    case 0: return launch<128, 128, 2, true, false, false, 256, 2, 0, 0, BNB, AX>(p, st);
    case 1: return launch<256, 64, 2, true, false, false, 256, 2, 0, 0, BNB, AX == 3 ? 2 : AX>(p, st);
    case 3: return launch<128, 64, 2, true, false, false, 256, 2, 0, 0, BNB, AX>(p, st);
    case 5: return launch<128, 128, 1, true, false, false, 256, 2, 0, 0, BNB, AX>(p, st);
    case 6: return launch<256, 64, 1, true, false, false, 256, 2, 0, 0, BNB, AX == 3 ? 2 : AX>(p, st);
    case 8: return launch<128, 64, 1, true, false, false, 256, 2, 0, 0, BNB, AX>(p, st);
    case 10: return launch<128, 128, 2, true, true, false, 256, 2, 0, 0, BNB, AX>(p, st);
    case 13: return launch<128, 64, 2, true, true, false, 256, 2, 0, 0, BNB, AX>(p, st);
    case 15: return launch<128, 128, 1, true, true, false, 256, 2, 0, 0, BNB, AX>(p, st);
    case 16: return launch<256, 64, 1, true, true, false, 256, 2, 0, 0, BNB, AX == 3 ? 2 : AX>(p, st);
    case 18: return launch<128, 64, 1, true, true, false, 256, 2, 0, 0, BNB, AX>(p, st);
    case 20: return launch<128, 128, 2, true, false, true, 256, 2, 0, 0, BNB, AX>(p, st);
    case 23: return launch<128, 64, 2, true, false, true, 256, 2, 0, 0, BNB, AX>(p, st);
    case 25: return launch<128, 128, 1, true, false, true, 256, 2, 0, 0, BNB, AX>(p, st);
    case 26: return launch<256, 64, 1, true, false, true, 256, 2, 0, 0, BNB, AX>(p, st);
    case 28: return launch<128, 64, 1, true, false, true, 256, 2, 0, 0, BNB, AX>(p, st);
    // the 8-wave 2-stage LDS-DMA tiles (64 x 64 per wave): one 256-row (128-row) workgroup tile
    // covers N = 128 (256) output channels, so an A row is applied by fewer column tiles
    case 30: return launch<256, 128, 2, true, false, true, 512, 4, 0, 0, BNB, AX>(p, st);
    case 31: return launch<128, 256, 2, true, false, true, 512, 2, 0, 0, BNB, AX>(p, st);
  }
  return -5;  // NOT_APPLICABLE: no AX instantiation of this tile
}

int launch_variant_ax(int v, const NTParams& p, hipStream_t st) {
  if (p.ax.mode == 1 && p.bnb.part == nullptr) return launch_ax<1, false>(v, p, st);
  if (p.ax.mode == 2 && p.bnb.part != nullptr) return launch_ax<2, true>(v, p, st);
  if (p.ax.mode == 3 && p.bnb.part != nullptr) return launch_ax<3, true>(v, p, st);
  return -5;
}

}  // namespace pdt_nt

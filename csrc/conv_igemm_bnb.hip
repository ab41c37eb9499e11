// Instantiations of the implicit-GEMM kernel (conv_nt_kernel.h) with the fused
// BatchNorm-backward epilogue (BNB = true): data gradients that also reduce
// the BN backward statistics of the unit they feed. A separate translation
// unit so these register-heavier epilogues neither change the plain kernels'
// register allocation nor serialise the build.
#include "conv_nt_kernel.h"

namespace pdt_nt {

int launch_variant_bnb(int v, bool cs64, const NTParams& p, hipStream_t st) {
  return cs64 ? launch_variant<true, true>(v, p, st) : launch_variant<false, true>(v, p, st);
}

int launch_variant_pers_bnb(int i, bool cs64, const NTParams& p, hipStream_t st) {
  return cs64 ? launch_variant_pers<true, true>(i, p, st) : launch_variant_pers<false, true>(i, p, st);
}

}  // namespace pdt_nt

// placeholder until the bf16 MFMA conv lands
#include "common.h"
namespace eosv {
int launch_conv_bf16(const ConvArgs&, hipStream_t) {
  set_error("conv_bf16: not implemented yet");
  return EOSV_ERR_UNSUPPORTED;
}
}  // namespace eosv

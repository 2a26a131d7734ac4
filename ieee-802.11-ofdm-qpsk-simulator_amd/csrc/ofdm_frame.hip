// ofdm_frame.hip -- frame mode: preambles, RRC, packet sync, CFO.
// (placeholder entry points; the kernels land in the next commit)
#include "ofdm_internal.h"
#include "ofdm_ctx.h"

using namespace ofdm;

extern "C" {

int ofdm_transmitter(ofdm_ctx *, int, int, int, float *, int32_t, int32_t *) {
    return set_error(OFDM_E_ARG, "frame mode not built yet");
}
int ofdm_transmission_over_air(ofdm_ctx *, const float *, float *, int32_t, double, uint64_t, uint64_t, int32_t) {
    return set_error(OFDM_E_ARG, "frame mode not built yet");
}
int ofdm_receiver(ofdm_ctx *, const float *, const ofdm_rx_opts *, int, float *, int32_t *, int32_t *, float *) {
    return set_error(OFDM_E_ARG, "frame mode not built yet");
}
int ofdm_frame_sweep(ofdm_ctx *, const ofdm_cfg *, const ofdm_rx_opts *, const double *, int, uint64_t, int64_t,
                     int64_t *, int32_t *) {
    return set_error(OFDM_E_ARG, "frame mode not built yet");
}

}  // extern "C"

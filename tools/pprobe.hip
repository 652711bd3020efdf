// Phase-timestamp build of the general kernel (diagnostic, not the product): the product
// source compiled with WTP_PROBE=1 as a separate shared library whose extra entry point
// points k_pieces' per-wave stamps at a caller buffer.  Driven by tools/pprobe.py.
#define WTP_PROBE 1
#include "../a3-reliable-transport_amd/csrc/crc32_kernels.hip"

extern "C" int pprobe_set(uint64_t *d_stamps) {
    return hipMemcpyToSymbol(HIP_SYMBOL(wtp::dev::g_probe), &d_stamps, sizeof(d_stamps)) == hipSuccess ? 0 : -1;
}

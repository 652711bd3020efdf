/*
 * wtp_diag.h — measurement probes (lib/libwtp_diag.so), used by bench.py and tools/.
 *
 * Not part of the drop-in boundary (wtp_crc32.h is): the reference has no counterpart.
 * They exist so a bench line can carry the same box's HBM read ceiling and clock next
 * to the CRC kernel's rate.
 */
#ifndef WTP_DIAG_H
#define WTP_DIAG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Streaming read of d_buf[0 .. nbytes & ~15) (nt dwordx4 loads, XOR-reduced; d_sink is
   written only for one improbable XOR value).  threads: multiple of 64, <= 512.
   Returns 0, or < 0 on a bad argument / launch failure.  Asynchronous on `stream`. */
int wtp_diag_read_xor(const void *d_buf, size_t nbytes, uint32_t *d_sink, unsigned blocks,
                      unsigned threads, void *stream);

/* One wave spins `iters` dependent VALU steps; d_out[0] = shader-clock ticks
   (s_memtime), d_out[1] = 100 MHz ticks (s_memrealtime) over the spin. */
int wtp_diag_clock(uint64_t *d_out, uint32_t iters, void *stream);

/* Timing-only HIP events (created with hipEventDisableSystemFence: no system-scope cache
   writeback/invalidate when recorded, so they perturb and pad the timed kernels least).
   elapsed_ms waits for `end`.  0 on success, < 0 on failure. */
int wtp_diag_event_create(void **ev);
int wtp_diag_event_record(void *ev, void *stream);
int wtp_diag_event_elapsed_ms(void *start, void *end, float *ms);
int wtp_diag_event_destroy(void *ev);
/* `stream` waits for event `ev` (hipStreamWaitEvent). */
int wtp_diag_stream_wait(void *stream, void *ev);

#ifdef __cplusplus
}
#endif

#endif /* WTP_DIAG_H */

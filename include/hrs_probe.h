/*
 * hrs_probe.h — HBM ceiling probes exported by libhrs.so (diagnostic; not part
 * of the codec plugin surface, so they have no reference counterpart).
 *
 * bench.py quotes the coding kernels' bandwidth against the nominal 8 TB/s
 * and against what this GPU streams in the same run ("a
 * measured device-copy STREAM peak"):
 *   - hrs_probe_stream: copy, read-only and write-only streams in the shapes
 *     of round 1's bandwidth lab (profiles/r01/lab8_bw_ceilings.txt): a wave
 *     task is `chunk_kib` KiB contiguous, one 16-byte access per lane per KiB,
 *     the task's loads all issued before any is used; nontemporal or default
 *     policy; bench.py takes the fastest of a small sweep of shapes.
 *   - hrs_probe_rows: the coding kernels' own access pattern with the GF math
 *     taken out. A 1:1 copy is not a ceiling for the codec's read-heavy mixes
 *     (RS(10,4) encode reads 10 rows per 4 written, a repair 10 per 1), and
 *     neither is the mix of the read-only and write-only peaks, because HBM
 *     pays for turning its bus between reads and writes; this probe moves the
 *     same bytes in the same order, so it is the ceiling of the pattern.
 * hrs_probe_copy / _read / _write are the 1 KiB-task nontemporal streams
 * (= a grid-stride loop over 16-byte elements).
 */
#ifndef HRS_PROBE_H_
#define HRS_PROBE_H_

#include <stddef.h>

#include "hrs.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { HRS_PROBE_COPY = 0, HRS_PROBE_READ = 1, HRS_PROBE_WRITE = 2 };

/* One streaming pass on `stream` (a hipStream_t; NULL = null stream),
 * asynchronous:
 *   HRS_PROBE_COPY  dst[0, bytes) = src[0, bytes);
 *   HRS_PROBE_READ  reads src[0, bytes) once; `dst` is a device sink of
 *                   >= 4 KiB, written only in a case that cannot occur (it
 *                   keeps the loads alive);
 *   HRS_PROBE_WRITE writes dst[0, bytes) once (src unused, may be NULL).
 * chunk_kib in {1, 2, 4, 8}: contiguous KiB per wave task; nontemporal != 0
 * uses nontemporal loads / stores; the grid is blocks_per_cu (1..32) x the
 * current device's CUs of 256 threads. Pointers and bytes must be multiples
 * of 16 (else HRS_EALIGN); other bad arguments HRS_EINVAL. */
hrs_status hrs_probe_stream(int op, const void* src, void* dst, size_t bytes, int chunk_kib, int nontemporal,
                            int blocks_per_cu, void* stream);

/* = hrs_probe_stream(HRS_PROBE_COPY, src, dst, bytes, 1, 1, blocks_per_cu, stream). */
hrs_status hrs_probe_copy(const void* src, void* dst, size_t bytes, int blocks_per_cu, void* stream);

/* = hrs_probe_stream(HRS_PROBE_READ, src, sink, bytes, 1, 1, blocks_per_cu, stream). */
hrs_status hrs_probe_read(const void* src, size_t bytes, int blocks_per_cu, void* sink, void* stream);

/* = hrs_probe_stream(HRS_PROBE_WRITE, NULL, dst, bytes, 1, 1, blocks_per_cu, stream). */
hrs_status hrs_probe_write(void* dst, size_t bytes, int blocks_per_cu, void* stream);

/* The coding kernels' access pattern without the math, over `nstripes`
 * stripes of `nrows` rows of `cell_bytes` each, stripe-major and contiguous
 * from `base` (the layout of encodeBulk's [parity..., data...] rows): per
 * 2 KiB column window, rows [nrows - nread, nrows) are read and rows
 * [0, nwrite) overwritten with their XOR (+ the row index). `schedule` sets
 * how the loads are spaced — D rows in flight per wave and M dependent VALU
 * steps per loaded dword in place of the GF math, since HBM serves a
 * spaced-out request stream better than a burst: 0 = all rows' loads first,
 * no math; 1 = D 3, M 12; 2 = D 5, M 6; 3 = D 1, M 0. cell_bytes must be a
 * multiple of 2048 and base of 16 (else HRS_EALIGN); (nread, nwrite) one of
 * (10,4) (10,3) (10,2) (10,1) (10,0) (6,3) (12,4) (12,2) (3,2), with
 * nread + nwrite <= nrows, schedule in [0, 3] (else HRS_EINVAL). Asynchronous
 * on `stream`. */
hrs_status hrs_probe_rows(void* base, size_t nstripes, int nrows, size_t cell_bytes, int nread, int nwrite,
                          int schedule, int blocks_per_cu, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* HRS_PROBE_H_ */

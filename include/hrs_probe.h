/*
 * hrs_probe.h — HBM ceiling probes, exported by libhrs_probe.so: a side
 * library that bench.py and tools load. The product library (libhrs.so, the
 * one a DataNode JVM loads) does not carry them; they have no reference
 * counterpart.
 *
 * bench.py quotes the coding kernels' bandwidth against the nominal 8 TB/s
 * and against what this GPU streams in the same run ("a
 * measured device-copy STREAM peak"):
 *   - hrs_probe_stream: copy, read-only and write-only streams under three
 *     schedules (tools/copy_lab.hip, profiles/r04/copy_lab/); bench.py takes
 *     the fastest of a small sweep;
 *   - hrs_probe_rows: the coding kernels' own access pattern with the GF math
 *     taken out. A 1:1 copy is not a ceiling for the codec's read-heavy mixes
 *     (RS(10,4) encode reads 10 rows per 4 written, a repair 10 per 1), and
 *     neither is the mix of the read-only and write-only peaks, because HBM
 *     pays for turning its bus between reads and writes; this probe moves the
 *     same bytes in the same order, so it is the ceiling of the pattern.
 */
#ifndef HRS_PROBE_H_
#define HRS_PROBE_H_

#include <stddef.h>

#include "hrs.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { HRS_PROBE_COPY = 0, HRS_PROBE_READ = 1, HRS_PROBE_WRITE = 2 };
enum { HRS_PROBE_WAVE_TASKS = 0, HRS_PROBE_GRID_STRIDE = 1, HRS_PROBE_BLOCK_RANGE = 2 };

/* One streaming pass over `bytes` on `stream` (a hipStream_t; NULL = null
 * stream), asynchronous:
 *   HRS_PROBE_COPY  dst[0, bytes) = src[0, bytes);
 *   HRS_PROBE_READ  reads src[0, bytes) once; `dst` is a device sink of
 *                   >= 4 KiB, written only if the data XOR to one particular
 *                   value (it keeps the loads alive);
 *   HRS_PROBE_WRITE writes dst[0, bytes) once (src unused, may be NULL).
 * schedule: HRS_PROBE_WAVE_TASKS — a wave task is `depth` contiguous KiB;
 * HRS_PROBE_GRID_STRIDE — thread i moves 16-byte elements i + j * (grid
 * threads), `depth` in flight; HRS_PROBE_BLOCK_RANGE — each block streams its
 * own contiguous 1/grid of the buffer, block-stride, `depth` elements per
 * thread in flight. depth in {1, 2, 4, 8}; in every schedule a thread issues
 * all `depth` loads before it uses one. nontemporal != 0 uses nontemporal
 * loads / stores. The grid is blocks_per_cu x the current device's CUs of
 * block_threads (256, 512 or 1024) threads, blocks_per_cu * block_threads <=
 * 8192. Pointers and bytes must be multiples of 16 (else HRS_EALIGN); other
 * bad arguments HRS_EINVAL. */
hrs_status hrs_probe_stream(int op, const void* src, void* dst, size_t bytes, int schedule, int depth,
                            int nontemporal, int block_threads, int blocks_per_cu, void* stream);

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

/*
 * hrs_probe.h — HBM ceiling probe exported by libhrs.so (diagnostic; not part
 * of the codec plugin surface, so it has no reference counterpart).
 *
 * bench.py quotes the coding kernels' bandwidth against the nominal 8 TB/s
 * and against what a plain streaming copy reaches on the same GPU in the same
 * run ("a measured device-copy STREAM peak"). The copy is
 * the shape MI355X_MICROARCH.md's STREAM figure uses — a grid-stride copy of
 * 16-byte elements, 256-thread blocks — with nontemporal loads and stores
 * (every byte moves once, like the codec's rows), at `blocks_per_cu` resident
 * blocks per CU (4 measured fastest on the pool, profiles/r02/copy_probe.json).
 *
 * A 1:1 copy is not a ceiling for the codec's read-heavy mixes (RS(10,4)
 * encode reads 10 rows per 4 written; a repair 10 per 1): HBM's data bus is
 * shared by reads and writes, so the read-only and write-only probes below
 * give the mix ceiling bench.py quotes, (R + W) / (R / read_peak +
 * W / write_peak) for R bytes read and W written.
 */
#ifndef HRS_PROBE_H_
#define HRS_PROBE_H_

#include <stddef.h>

#include "hrs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* dst[0, bytes) = src[0, bytes) on `stream` (a hipStream_t; NULL = null
 * stream), asynchronous. src, dst and bytes must be multiples of 16 (else
 * HRS_EALIGN); blocks_per_cu in [1, 32] (else HRS_EINVAL). The grid is
 * blocks_per_cu x the current device's CUs. */
hrs_status hrs_probe_copy(const void* src, void* dst, size_t bytes, int blocks_per_cu, void* stream);

/* Reads src[0, bytes) once (nontemporal 16-byte loads, same grid shape);
 * `sink` is a device buffer of >= 4 KiB that is written only in a case that
 * cannot occur (it keeps the loads alive). */
hrs_status hrs_probe_read(const void* src, size_t bytes, int blocks_per_cu, void* sink, void* stream);

/* Writes dst[0, bytes) once (nontemporal 16-byte stores, same grid shape). */
hrs_status hrs_probe_write(void* dst, size_t bytes, int blocks_per_cu, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* HRS_PROBE_H_ */

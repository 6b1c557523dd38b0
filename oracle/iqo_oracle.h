/*
 * iqo_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of libiqo's `*ResizerImpl<ArchGeneric>` (the bit-exact oracle for the
 * Lanczos / Area / Linear U8 resize hot path).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker / the timed
 * CPU baseline.  The product (libiqo_amd) never links or calls it.
 *
 * Parity is pinned by tests/golden/ (vectors produced by the reference's own Generic TUs,
 * compiled from /root/reference by oracle/Makefile into oracle/_ref/).
 */
#ifndef IQO_ORACLE_H
#define IQO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { IQO_ORACLE_LANCZOS = 0, IQO_ORACLE_AREA = 1, IQO_ORACLE_LINEAR = 2 };

/* Opaque resizer state (tables + work row); mirrors one I*ResizerImpl instance. */
typedef struct iqo_oracle iqo_oracle;

/* Construct: same arguments as the reference constructors (degree/pxScale ignored for area/linear).
 * Returns NULL on invalid sizes (zero) or allocation failure. */
iqo_oracle *iqo_oracle_new(int method, unsigned degree, size_t srcW, size_t srcH,
                           size_t dstW, size_t dstH, size_t pxScale);
void iqo_oracle_free(iqo_oracle *o);

/* resize(srcSt, src, dstSt, dst) -- same semantics as I*ResizerImpl::resize. */
void iqo_oracle_resize(iqo_oracle *o, size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst);

/* Table introspection: axis 0 = X, 1 = Y.  Writes nTaps*nPhases values (int16 or u16 bit
 * pattern widened to int32) if cap allows; returns nTaps*nPhases or -1. */
int iqo_oracle_table(const iqo_oracle *o, int axis, int *nTaps, int *nPhases, int32_t *buf, size_t cap);

/* One-shot convenience. Returns 0 on success. */
int iqo_oracle_run(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                   size_t pxScale, size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst);

/* CPU baseline: resize nFrames frames (frame strides in bytes) with nThreads std-thread-style
 * workers (pthreads), one oracle instance per worker (instances are not re-entrant, exactly like
 * the reference's Generic impl).  Returns elapsed seconds (wall clock, CLOCK_MONOTONIC). */
double iqo_oracle_run_batch(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW,
                            size_t dstH, size_t pxScale, size_t nFrames, size_t srcSt,
                            size_t srcFrameSt, const uint8_t *src, size_t dstSt, size_t dstFrameSt,
                            uint8_t *dst, int nThreads);

/* Input generators shared by tests and bench (defined precisely so numpy/GPU can match). */
void iqo_gen_g1(uint8_t *p, size_t w, size_t h, size_t st);            /* (i*2654435761)>>24 */
void iqo_gen_mt19937(uint8_t *p, size_t n, uint32_t seed);             /* benchmark.cpp fillRandom */
void iqo_gen_splitmix(uint8_t *p, size_t n, uint64_t seed);            /* noise */

uint64_t iqo_fnv1a64(const uint8_t *p, size_t w, size_t h, size_t st);

#ifdef __cplusplus
}
#endif
#endif

// covt_internal.h -- declarations shared by the kernel and host translation units of libcovt.
#ifndef COVT_INTERNAL_H
#define COVT_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "covt.h"

#ifdef __cplusplus
extern "C" {
#endif

// Enqueues the one-wave-per-stream decode kernel of one codec family (covt_decode.hip) on `stream`
// over descriptors [0, n_streams); descriptors of other families are skipped.
int covt_launch_family(int fam, const uint8_t* d_in, const covt_stream_desc* d_desc, int64_t n_streams,
                       uint8_t* d_out, covt_stream_result* d_res, hipStream_t stream);
int covt_op_family_of(int op);

#ifdef __cplusplus
}
#endif
#endif

/*
 * vbhem_dist.h -- the one collective of a sharded EM run: a SUM
 * all-reduce of the packed K-cluster statistics (vbhem_estep_fused's vector) over
 * RCCL, issued in-stream by the C++ EM loop (vbhem_em_run_ext) or by a caller.
 *
 * Reference: the reduction over base HMMs i of vbhem_compute_Statistics.m:44-50,
 * called per cluster at vbhem_h3m_c_step_fc.m:400-419.  With the bases sharded over
 * G GPUs (one process per GPU) each rank sums its own shard; this call adds the
 * G partial vectors.
 *
 * RCCL is resolved at run time: the instance already in the process (the
 * librccl.so that PyTorch loads) when there is one, else librccl.so.1 from
 * /opt/rocm/lib.  Status codes as in vbhem_estep.h (VBHEM_ERR_HIP also covers
 * RCCL errors; vbhem_last_error() names them).
 */
#ifndef VBHEM_DIST_H
#define VBHEM_DIST_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VBHEM_RCCL_ID_BYTES 128 /* NCCL_UNIQUE_ID_BYTES */

/* VBHEM_OK when RCCL can be bound in this process (else VBHEM_ERR_UNSUPPORTED):
 * every rank checks it, and the ranks agree on the result, before any of them
 * enters the collective initialisation (a rank that cannot would leave the others
 * waiting inside ncclCommInitRank). */
int vbhem_rccl_available(void);

/* A communicator id (rank 0 makes it, the caller hands the bytes to every rank). */
int vbhem_rccl_unique_id(void *id /* [VBHEM_RCCL_ID_BYTES] */);

/* ncclCommInitRank on `device` (made current for the call); *comm receives the
 * communicator. */
int vbhem_rccl_comm_init(int nranks, int rank, const void *id, int device, void **comm);

int vbhem_rccl_comm_destroy(void *comm);

/* In-place SUM all-reduce of n doubles on `stream` (asynchronous). */
int vbhem_rccl_allreduce_sum(void *comm, double *buf, size_t n, void *stream);

/* The same, then the reduced vector copied by a kernel on `stream` into out_dev: the
 * device address of pinned host memory (vbhem_host_device_pointer), where the host
 * M-step reads it after one event -- as the one-rank fused call's statistics kernel
 * writes it there -- with no hipMemcpy between the E-steps of a paced loop. */
int vbhem_rccl_allreduce_to(void *comm, double *buf, size_t n, double *out_dev, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* VBHEM_DIST_H */

/*
 * status.h -- return codes of the C ABI.
 *
 * The reference primitives are `void` and report nothing: mismatched counts
 * or ports deadlock and tests rely on timeouts (test/reduce/test_reduce.cpp:
 * 34-46); an invalid reduce type/op is a code-generator assert
 * (codegen/ops.py:146-147).  Every entry point here returns one of these
 * codes instead; the Python mirror raises on any non-zero code.
 */
#ifndef SMI_STATUS_H
#define SMI_STATUS_H

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    SMI_SUCCESS = 0,
    SMI_ERR_INVALID_ARG = -1,     /* bad size, null pointer, misalignment  */
    SMI_ERR_UNSUPPORTED = -2,     /* type/op combination not provided      */
    SMI_ERR_HIP = -3,             /* a HIP runtime call failed             */
    SMI_ERR_COMM = -4,            /* RCCL / transport failure              */
    SMI_ERR_BAD_COMM = -5,        /* unknown or finalized communicator     */
    SMI_ERR_NO_DEVICE = -6        /* no GPU visible                        */
} SMI_Status;

/* Human-readable text for the last error raised on the calling thread. */
const char *smi_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SMI_STATUS_H */

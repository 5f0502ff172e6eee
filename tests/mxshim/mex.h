/*
 * tests/mxshim/mex.h -- TEST DOUBLE of the subset of MATLAB's MEX/mx C API that
 * integration/vbhem_hmm_bwd_fwd_mex.c uses.  MATLAB is not available in this
 * image; in a MATLAB installation the gateway is compiled with `mex` against
 * MATLAB's own mex.h/libmx instead.  Only our own gateway is
 * built against this file; the reference MEX is not.
 */
#ifndef VBHEM_TEST_MEX_H
#define VBHEM_TEST_MEX_H
#include <stdbool.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mxArray_tag mxArray;
typedef size_t mwSize;
typedef size_t mwIndex;
typedef enum { mxUNKNOWN_CLASS = 0, mxCELL_CLASS, mxSTRUCT_CLASS, mxDOUBLE_CLASS } mxClassID;
typedef enum { mxREAL = 0, mxCOMPLEX } mxComplexity;

mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray *mxCreateDoubleScalar(double v);
mxArray *mxCreateNumericArray(mwSize ndim, const mwSize *dims, mxClassID cls, mxComplexity c);
mxArray *mxCreateCellMatrix(mwSize m, mwSize n);
mxArray *mxCreateStructMatrix(mwSize m, mwSize n, int nfields, const char **fieldnames);
void mxDestroyArray(mxArray *a);
mxArray *mxGetCell(const mxArray *a, mwIndex i);
void mxSetCell(mxArray *a, mwIndex i, mxArray *v);
mxArray *mxGetField(const mxArray *a, mwIndex i, const char *name);
void mxSetField(mxArray *a, mwIndex i, const char *name, mxArray *v);
double *mxGetPr(const mxArray *a);
double mxGetScalar(const mxArray *a);
mwSize mxGetM(const mxArray *a);
mwSize mxGetN(const mxArray *a);
mwSize mxGetNumberOfElements(const mxArray *a);
mwSize mxGetNumberOfDimensions(const mxArray *a);
const mwSize *mxGetDimensions(const mxArray *a);
bool mxIsCell(const mxArray *a);
bool mxIsStruct(const mxArray *a);
bool mxIsDouble(const mxArray *a);
bool mxIsComplex(const mxArray *a);
void *mxMalloc(size_t n);
void *mxCalloc(size_t n, size_t sz);
void mxFree(void *p);
void mexErrMsgIdAndTxt(const char *id, const char *fmt, ...);
int mexPrintf(const char *fmt, ...);
int mexAtExit(void (*fn)(void));

/* the gateway entry point MATLAB calls */
void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]);

#ifdef __cplusplus
}
#endif
#endif

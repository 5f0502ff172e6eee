/*
 * tests/mxshim/mxshim.c -- TEST DOUBLE of MATLAB's mx/mex runtime (see mex.h).
 * Column-major double arrays, cells and structs; mexErrMsgIdAndTxt unwinds to
 * mxshim_call() with longjmp, the way MATLAB aborts a MEX call.  Arrays are
 * never freed automatically (tests call mxDestroyArray).
 */
#include "mex.h"

#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct mxArray_tag {
  mxClassID cls;
  mwSize ndim;
  mwSize dims[8];
  mwSize numel;
  double *pr;          /* double */
  mxArray **cells;     /* cell / struct field values (numel * nfields) */
  int nfields;
  char **fieldnames;
};

static jmp_buf g_jmp;
static int g_in_call = 0;
static char g_err_id[256];
static char g_err_msg[1024];

static mxArray *alloc_array(mxClassID cls, mwSize ndim, const mwSize *dims) {
  mxArray *a = (mxArray *)calloc(1, sizeof(mxArray));
  a->cls = cls;
  a->ndim = ndim < 2 ? 2 : ndim;
  a->numel = 1;
  for (mwSize k = 0; k < a->ndim; k++) {
    a->dims[k] = k < ndim ? dims[k] : 1;
    a->numel *= a->dims[k];
  }
  return a;
}

mxArray *mxCreateNumericArray(mwSize ndim, const mwSize *dims, mxClassID cls, mxComplexity c) {
  (void)c;
  mxArray *a = alloc_array(cls, ndim, dims);
  a->pr = (double *)calloc(a->numel ? a->numel : 1, sizeof(double));
  return a;
}

mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) {
  mwSize d[2] = {m, n};
  return mxCreateNumericArray(2, d, mxDOUBLE_CLASS, c);
}

mxArray *mxCreateDoubleScalar(double v) {
  mxArray *a = mxCreateDoubleMatrix(1, 1, mxREAL);
  a->pr[0] = v;
  return a;
}

mxArray *mxCreateCellMatrix(mwSize m, mwSize n) {
  mwSize d[2] = {m, n};
  mxArray *a = alloc_array(mxCELL_CLASS, 2, d);
  a->cells = (mxArray **)calloc(a->numel ? a->numel : 1, sizeof(mxArray *));
  return a;
}

mxArray *mxCreateStructMatrix(mwSize m, mwSize n, int nfields, const char **fieldnames) {
  mwSize d[2] = {m, n};
  mxArray *a = alloc_array(mxSTRUCT_CLASS, 2, d);
  a->nfields = nfields;
  a->fieldnames = (char **)calloc(nfields ? nfields : 1, sizeof(char *));
  for (int f = 0; f < nfields; f++) a->fieldnames[f] = strdup(fieldnames[f]);
  a->cells = (mxArray **)calloc((a->numel ? a->numel : 1) * (nfields ? nfields : 1), sizeof(mxArray *));
  return a;
}

void mxDestroyArray(mxArray *a) {
  if (!a) return;
  if (a->cls == mxCELL_CLASS)
    for (mwSize k = 0; k < a->numel; k++) mxDestroyArray(a->cells[k]);
  if (a->cls == mxSTRUCT_CLASS) {
    for (mwSize k = 0; k < a->numel * (mwSize)a->nfields; k++) mxDestroyArray(a->cells[k]);
    for (int f = 0; f < a->nfields; f++) free(a->fieldnames[f]);
    free(a->fieldnames);
  }
  free(a->cells);
  free(a->pr);
  free(a);
}

mxArray *mxGetCell(const mxArray *a, mwIndex i) {
  return (a && a->cls == mxCELL_CLASS && i < a->numel) ? a->cells[i] : NULL;
}

void mxSetCell(mxArray *a, mwIndex i, mxArray *v) {
  if (a && a->cls == mxCELL_CLASS && i < a->numel) a->cells[i] = v;
}

static int field_index(const mxArray *a, const char *name) {
  for (int f = 0; f < a->nfields; f++)
    if (strcmp(a->fieldnames[f], name) == 0) return f;
  return -1;
}

mxArray *mxGetField(const mxArray *a, mwIndex i, const char *name) {
  if (!a || a->cls != mxSTRUCT_CLASS || i >= a->numel) return NULL;
  int f = field_index(a, name);
  return f < 0 ? NULL : a->cells[i * a->nfields + f];
}

void mxSetField(mxArray *a, mwIndex i, const char *name, mxArray *v) {
  if (!a || a->cls != mxSTRUCT_CLASS || i >= a->numel) return;
  int f = field_index(a, name);
  if (f >= 0) a->cells[i * a->nfields + f] = v;
}

double *mxGetPr(const mxArray *a) { return a ? a->pr : NULL; }
double mxGetScalar(const mxArray *a) { return (a && a->pr && a->numel) ? a->pr[0] : 0.0; }
mwSize mxGetM(const mxArray *a) { return a ? a->dims[0] : 0; }
mwSize mxGetN(const mxArray *a) {
  if (!a) return 0;
  mwSize n = 1;
  for (mwSize k = 1; k < a->ndim; k++) n *= a->dims[k];
  return n;
}
mwSize mxGetNumberOfElements(const mxArray *a) { return a ? a->numel : 0; }
mwSize mxGetNumberOfDimensions(const mxArray *a) { return a ? a->ndim : 0; }
const mwSize *mxGetDimensions(const mxArray *a) { return a ? a->dims : NULL; }
bool mxIsCell(const mxArray *a) { return a && a->cls == mxCELL_CLASS; }
bool mxIsStruct(const mxArray *a) { return a && a->cls == mxSTRUCT_CLASS; }
bool mxIsDouble(const mxArray *a) { return a && a->cls == mxDOUBLE_CLASS; }
bool mxIsComplex(const mxArray *a) { (void)a; return false; }
void *mxMalloc(size_t n) { return malloc(n ? n : 1); }
void *mxCalloc(size_t n, size_t sz) { return calloc(n ? n : 1, sz ? sz : 1); }
void mxFree(void *p) { free(p); }

void mexErrMsgIdAndTxt(const char *id, const char *fmt, ...) {
  va_list ap;
  snprintf(g_err_id, sizeof(g_err_id), "%s", id ? id : "");
  va_start(ap, fmt);
  vsnprintf(g_err_msg, sizeof(g_err_msg), fmt, ap);
  va_end(ap);
  if (g_in_call) longjmp(g_jmp, 1);
  fprintf(stderr, "mexErrMsgIdAndTxt outside mxshim_call: %s: %s\n", g_err_id, g_err_msg);
  abort();
}

int mexPrintf(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  int n = vprintf(fmt, ap);
  va_end(ap);
  return n;
}

/* ---- test-harness helpers (not part of the MATLAB API) ------------------------- */
/* MATLAB runs the registered function when the MEX file is cleared; the double
   runs it from mxshim_clear() */
static void (*g_atexit)(void) = NULL;
int mexAtExit(void (*fn)(void)) {
  g_atexit = fn;
  return 0;
}
void mxshim_clear(void) {
  if (g_atexit) g_atexit();
}

typedef void (*mex_fn)(int, mxArray **, int, const mxArray **);

/* Returns 0 on success, 1 if the gateway raised mexErrMsgIdAndTxt. */
int mxshim_call(mex_fn fn, int nlhs, mxArray **plhs, int nrhs, const mxArray **prhs) {
  g_err_id[0] = g_err_msg[0] = 0;
  g_in_call = 1;
  if (setjmp(g_jmp)) {
    g_in_call = 0;
    return 1;
  }
  fn(nlhs, plhs, nrhs, prhs);
  g_in_call = 0;
  return 0;
}

const char *mxshim_error_id(void) { return g_err_id; }
const char *mxshim_error_msg(void) { return g_err_msg; }

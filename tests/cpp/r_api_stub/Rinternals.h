/* Declarations-only stand-in of the few R API items rpkg/src/nngp_shim.c
 * uses, for a compile (syntax + type) check of the shim in this image, which
 * has no R.  Test infrastructure: the shim is built against R's real headers
 * by `R CMD INSTALL rpkg` where R exists. */
#ifndef R_API_STUB_RINTERNALS_H
#define R_API_STUB_RINTERNALS_H
#include <stddef.h>
typedef struct SEXPREC* SEXP;
typedef ptrdiff_t R_xlen_t;
typedef unsigned char Rbyte;
typedef int Rboolean;
#define TRUE 1
#define FALSE 0
enum { NILSXP = 0, INTSXP = 13, REALSXP = 14, STRSXP = 16, VECSXP = 19, EXTPTRSXP = 22, RAWSXP = 24 };
extern SEXP R_NilValue, R_NamesSymbol;
int TYPEOF(SEXP);
double* REAL(SEXP);
int* INTEGER(SEXP);
Rbyte* RAW(SEXP);
R_xlen_t XLENGTH(SEXP);
SEXP VECTOR_ELT(SEXP, R_xlen_t);
SEXP SET_VECTOR_ELT(SEXP, R_xlen_t, SEXP);
void SET_STRING_ELT(SEXP, R_xlen_t, SEXP);
SEXP Rf_allocVector(int, R_xlen_t);
SEXP Rf_allocMatrix(int, int, int);
SEXP Rf_protect(SEXP);
void Rf_unprotect(int);
#define PROTECT(s) Rf_protect(s)
#define UNPROTECT(n) Rf_unprotect(n)
int Rf_nrows(SEXP);
int Rf_ncols(SEXP);
Rboolean Rf_isMatrix(SEXP);
int Rf_asInteger(SEXP);
double Rf_asReal(SEXP);
SEXP Rf_ScalarInteger(int);
SEXP Rf_ScalarReal(double);
SEXP Rf_mkString(const char*);
SEXP Rf_mkChar(const char*);
SEXP Rf_install(const char*);
SEXP Rf_setAttrib(SEXP, SEXP, SEXP);
void Rf_error(const char*, ...);
SEXP R_MakeExternalPtr(void*, SEXP, SEXP);
void* R_ExternalPtrAddr(SEXP);
SEXP R_ExternalPtrTag(SEXP);
SEXP R_ExternalPtrProtected(SEXP);
void R_SetExternalPtrProtected(SEXP, SEXP);
void R_ClearExternalPtr(SEXP);
typedef void (*R_CFinalizer_t)(SEXP);
void R_RegisterCFinalizerEx(SEXP, R_CFinalizer_t, Rboolean);
#endif

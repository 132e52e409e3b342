/* see Rinternals.h in this directory (compile check of the R shim only) */
#include <stdio.h>

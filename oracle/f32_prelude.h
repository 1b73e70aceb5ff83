/* Float restatement of the oracle (TEST INFRASTRUCTURE, fp32 floor study only; tools/fp32_floor.py --float-oracle).
 * Force-included before every oracle source by `make liboracle_f32.so`: the system headers are pulled in first
 * (their include guards make the sources' own includes no-ops), then every `double` of the oracle becomes `float`
 * -- the same algorithm, statement for statement, in single precision (libm calls still round once to float).
 * Never linked into the product or the default oracle. */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define double float

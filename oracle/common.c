/*
 * CPU ORACLE (test infrastructure only; see oracle.h).
 * Thread control for the OpenMP loops (the reference's own CPU path is
 * parallel through OpenCV parallel_for_ / std::thread, batch.cpp:181-200).
 */
#include "oracle.h"
#include <omp.h>

void orc_set_threads(int n) { if (n > 0) omp_set_num_threads(n); }
int orc_get_threads(void) { return omp_get_max_threads(); }

/* A plain C99 consumer of include/gcg_spmm.h (no HIP headers, no Python): what a C/C++ or
 * cgo/JNI binding would compile against. Exercises the host-only planner and the status
 * protocol; the device entry points are exercised by the GPU tests. */
#include <stdio.h>
#include <string.h>

#include "gcg_spmm.h"

int main(void) {
  /* rows: 3 nnz, 1 nnz, 700 nnz, 0 nnz */
  int32_t indptr[5] = {0, 3, 4, 704, 704};
  int64_t n_tasks = 0, n_long = 0, n_slots = 0;
  gcg_status st = gcg_spmm_plan_host(4, indptr, NULL, 0, 256, 0, NULL, 0, &n_tasks, NULL, 0,
                                     &n_long, &n_slots);
  if (st != GCG_OK) { printf("plan sizing failed: %s\n", gcg_last_error()); return 1; }
  int32_t tasks[64 * 4], longs[16 * 4];
  if (n_tasks > 64 || n_long > 16) return 2;
  st = gcg_spmm_plan_host(4, indptr, NULL, 0, 256, 0, tasks, 64, &n_tasks, longs, 16, &n_long,
                          &n_slots);
  if (st != GCG_OK) return 3;
  /* row 2 (700 nnz) splits into 3 segments; rows 0-1 and row 3 are short tasks */
  if (n_long != 1 || n_slots != 3 || longs[0] != 2 || longs[2] != 3) return 4;
  int32_t bad[3] = {0, 5, 3};
  st = gcg_spmm_plan_host(2, bad, NULL, 0, 0, 0, NULL, 0, &n_tasks, NULL, 0, &n_long, &n_slots);
  if (st != GCG_ERR_BAD_CSR || strlen(gcg_last_error()) == 0) return 5;
  printf("abi ok: version %s, %lld tasks, %lld split rows\n", gcg_version(), (long long)n_tasks,
         (long long)n_long);
  return 0;
}

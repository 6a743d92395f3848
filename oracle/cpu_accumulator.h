/*
 * cpu_accumulator.h — CPU restatement of NodeNUMAResource's CPU accumulator (takeCPUs).
 * TEST INFRASTRUCTURE ONLY (see koord_oracle.c).
 */
#pragma once
#include <stdint.h>

#define KO_MAX_CPUS 256

enum { KO_EXCL_NONE = 0, KO_EXCL_PCPU = 1, KO_EXCL_NUMA = 2 };  /* CPUExclusivePolicy */
enum { KO_BIND_FULL_PCPUS = 1, KO_BIND_SPREAD_BY_PCPUS = 2 };    /* CPUBindPolicy */
enum { KO_NUMA_MOST = 0, KO_NUMA_LEAST = 1 };                    /* NUMAAllocateStrategy */

/* CPUTopology (cpu_topology.go:27-33): CPU i has core / NUMA node / socket ids; CPU ids are 0..ncpus-1 */
typedef struct ko_topo {
  int ncpus;
  int core[KO_MAX_CPUS], node[KO_MAX_CPUS], socket[KO_MAX_CPUS];
  int num_cores, num_nodes, num_sockets; /* distinct ids (CPUTopologyBuilder counts) */
} ko_topo;

/* fills num_* from the per-CPU ids */
void ko_topo_finish(ko_topo *t);

/* takeCPUs (cpu_accumulator.go:86-232).  avail[c] = c is in availableCPUs; refcount[c] / excl[c] =
 * allocatedCPUs[c].RefCount / ExclusivePolicy (excl[c] < 0: c not allocated).  out[c] = 1 for the CPUs
 * taken.  Returns 0, or -1 for the reference's error returns. */
int ko_take_cpus(const ko_topo *t, int max_ref, const uint8_t *avail, const int32_t *refcount, const int8_t *excl,
                 int needed, int bind, int excl_policy, int strategy, uint8_t *out);

/* acc.spreadCPUs(acc.freeCPUs(false)) on an empty node (TestCPUSpreadByPCPUs); returns the count */
int ko_spread_order(const ko_topo *t, int strategy, int *order);

#include <stdio.h>
#include <stddef.h>
#include "koordgpu.h"
#define P(T) printf("%s %zu\n", #T, sizeof(T))
#define O(T, f) printf("%s.%s %zu\n", #T, #f, offsetof(T, f))
int main(void) {
  P(ks_fit_args); P(ks_loadaware_args); P(ks_quota_args); P(ks_config); P(ks_node_cols); P(ks_pod_cols);
  P(ks_quota_cols); P(ks_quota_tree); P(ks_result); P(ks_node_state); P(ks_stats);
  P(ks_reservation_args); P(ks_reservation_cols);
  O(ks_config, fit); O(ks_config, loadaware); O(ks_config, quota); O(ks_config, batch_pods); O(ks_config, profile);
  O(ks_node_cols, alloc_scalar); O(ks_node_cols, la_flags); O(ks_node_cols, la_prod_usage_milli_memory);
  O(ks_pod_cols, flags); O(ks_pod_cols, quota_req); O(ks_quota_cols, nonpreemptible_used);
  O(ks_quota_tree, max); O(ks_quota_tree, self_request); O(ks_quota_tree, cluster_total); O(ks_stats, sweep_ms); O(ks_stats, diag);
  O(ks_config, reservation); O(ks_pod_cols, rsv_class); O(ks_result, reservation); O(ks_reservation_cols, allocatable);
  O(ks_reservation_cols, allocated); O(ks_reservation_cols, assigned); O(ks_reservation_cols, reserve_nonzero_memory);
  P(ks_numa_args); P(ks_deviceshare_args); P(ks_device_cols); P(ks_cpu_topology); P(ks_cpu_state_cols);
  O(ks_config, numa); O(ks_config, deviceshare); O(ks_numa_args, numa_scoring_strategy); O(ks_pod_cols, gpu_core);
  O(ks_pod_cols, cpu_bind); O(ks_cpu_topology, numa_node); O(ks_cpu_topology, socket); O(ks_cpu_state_cols, reserved);
  O(ks_node_cols, numa_flags); O(ks_result, gpu_minors);
  P(ks_numa_node_cols); O(ks_numa_node_cols, used_present); O(ks_numa_node_cols, cpuset_cpus);
  P(ks_node_pod_cols); O(ks_node_pod_cols, req_scalar); O(ks_node_pod_cols, quota_req); P(ks_preempt_result);
  O(ks_preempt_result, potential_nodes);
  return 0;
}

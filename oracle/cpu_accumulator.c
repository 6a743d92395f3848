/*
 * cpu_accumulator.c — CPU restatement of NodeNUMAResource's CPU accumulator.
 *
 * TEST INFRASTRUCTURE ONLY (parity oracle; see koord_oracle.c).  Follows
 * pkg/scheduler/plugins/nodenumaresource/cpu_accumulator.go:
 *   takeCPUs :86-232, newCPUAccumulator :247-286, take :288-302, needs / isSatisfied / isFailed :304-314,
 *   extractCPU :330-341, sortCores :343-367, freeCoresInNode :370-455, freeCoresInSocket :458-519,
 *   freeCPUsInNode :522-595, freeCPUsInSocket :598-640, freeCPUs :650-770, getCoreRefCount :772-779,
 *   sortCPUsByRefCount :781-792, spreadCPUs :794-822.
 * Go maps become per-id arrays; every sort.Slice here has a total order except the two
 * len-only sorts of the FullPCPUs fallback, where Go's insertion sort (n <= 12 sockets) is stable —
 * restated with a stable insertion sort.
 */
#include "cpu_accumulator.h"

#include <string.h>

#define N KO_MAX_CPUS

typedef struct acc {
  const ko_topo *t;
  int max_ref;
  uint8_t alloc[N];  /* allocatableCPUs */
  int32_t ref[N];    /* RefCount of allocatable CPUs (maxRefCount > 1 only) */
  int excl_cores[N], n_excl_cores;
  int excl_nodes[N], n_excl_nodes;
  int exclusive, excl_policy, strategy, needed;
  uint8_t result[N];
} acc_t;

/* a list of groups over one flat CPU array: group g = cpus[beg[g] .. beg[g]+len[g]) with key id[g] */
typedef struct groups {
  int cpus[N];
  int beg[N], len[N], id[N];
  int n;
} groups_t;

static int has(const int *s, int n, int v) {
  for (int i = 0; i < n; ++i)
    if (s[i] == v) return 1;
  return 0;
}

void ko_topo_finish(ko_topo *t) {
  /* CPUTopologyBuilder counts (cpu_topology.go:45-70): sockets, (socket, node) pairs, (socket, node, core) triples */
  int socks[N], ns = 0;
  int np_s[N], np_n[N], npair = 0;
  int nt_s[N], nt_n[N], nt_c[N], ntri = 0;
  for (int c = 0; c < t->ncpus; ++c) {
    if (!has(socks, ns, t->socket[c])) socks[ns++] = t->socket[c];
    int f = 0;
    for (int i = 0; i < npair; ++i) f |= np_s[i] == t->socket[c] && np_n[i] == t->node[c];
    if (!f) { np_s[npair] = t->socket[c]; np_n[npair] = t->node[c]; ++npair; }
    f = 0;
    for (int i = 0; i < ntri; ++i) f |= nt_s[i] == t->socket[c] && nt_n[i] == t->node[c] && nt_c[i] == t->core[c];
    if (!f) { nt_s[ntri] = t->socket[c]; nt_n[ntri] = t->node[c]; nt_c[ntri] = t->core[c]; ++ntri; }
  }
  t->num_sockets = ns;
  t->num_nodes = npair;
  t->num_cores = ntri;
}

static int cpus_per_core(const ko_topo *t) { return t->num_cores ? t->ncpus / t->num_cores : 0; }
static int cpus_per_socket(const ko_topo *t) { return t->num_sockets ? t->ncpus / t->num_sockets : 0; }
static int cpus_per_node(const ko_topo *t) { return t->num_nodes ? t->ncpus / t->num_nodes : 0; }

/* strategy order of two free counts: NUMAMostAllocated ascending, otherwise descending; 0 = tie */
static int strat_cmp(const acc_t *a, int x, int y) {
  if (x == y) return 0;
  if (a->strategy == KO_NUMA_MOST) return x < y ? -1 : 1;
  return x > y ? -1 : 1;
}

static int n_alloc(const acc_t *a) {
  int k = 0;
  for (int c = 0; c < a->t->ncpus; ++c) k += a->alloc[c];
  return k;
}

static void take(acc_t *a, const int *cpus, int n) {
  for (int i = 0; i < n; ++i) {
    const int c = cpus[i];
    a->result[c] = 1;
    a->alloc[c] = 0;
    if (a->exclusive) {
      if (a->excl_policy == KO_EXCL_PCPU && !has(a->excl_cores, a->n_excl_cores, a->t->core[c]))
        a->excl_cores[a->n_excl_cores++] = a->t->core[c];
      else if (a->excl_policy == KO_EXCL_NUMA && !has(a->excl_nodes, a->n_excl_nodes, a->t->node[c]))
        a->excl_nodes[a->n_excl_nodes++] = a->t->node[c];
    }
  }
  a->needed -= n;
}

static int needs(const acc_t *a, int n) { return a->needed >= n; }
static int satisfied(const acc_t *a) { return a->needed < 1; }

static int excl_pcpu(const acc_t *a, int c) {
  return a->excl_policy == KO_EXCL_PCPU && has(a->excl_cores, a->n_excl_cores, a->t->core[c]);
}
static int excl_numa(const acc_t *a, int c) {
  return a->excl_policy == KO_EXCL_NUMA && has(a->excl_nodes, a->n_excl_nodes, a->t->node[c]);
}

static void sort_ints(int *v, int n) {
  for (int i = 1; i < n; ++i) {
    const int x = v[i];
    int j = i - 1;
    while (j >= 0 && v[j] > x) { v[j + 1] = v[j]; --j; }
    v[j + 1] = x;
  }
}

/* sortCPUsByRefCount: refcount asc, cpu asc */
static void sort_by_ref(const acc_t *a, int *v, int n) {
  for (int i = 1; i < n; ++i) {
    const int x = v[i];
    int j = i - 1;
    while (j >= 0 && (a->ref[v[j]] > a->ref[x] || (a->ref[v[j]] == a->ref[x] && v[j] > x))) { v[j + 1] = v[j]; --j; }
    v[j + 1] = x;
  }
}

static int core_ref(const acc_t *a, int core) {
  int r = 0;
  for (int c = 0; c < a->t->ncpus; ++c)
    if (a->alloc[c] && a->t->core[c] == core) r += a->ref[c];
  return r;
}

/* cpus of the allocatable set grouped by core (first-seen order by CPU id), with a per-CPU filter */
typedef struct cores {
  int id[N], n_cpus[N], cpus[N][8];
  int n;
} cores_t;

static int core_slot(cores_t *cs, int core) {
  for (int i = 0; i < cs->n; ++i)
    if (cs->id[i] == core) return i;
  cs->id[cs->n] = core;
  cs->n_cpus[cs->n] = 0;
  return cs->n++;
}

/* sortCores: CPU count desc, (core refcount asc), core id asc — over slot indices */
static void sort_cores(const acc_t *a, const cores_t *cs, int *slots, int n) {
  for (int i = 1; i < n; ++i) {
    const int x = slots[i];
    int j = i - 1;
    for (; j >= 0; --j) {
      const int y = slots[j];
      int before; /* x before y? */
      if (cs->n_cpus[x] != cs->n_cpus[y]) before = cs->n_cpus[x] > cs->n_cpus[y];
      else if (a->max_ref > 1 && core_ref(a, cs->id[x]) != core_ref(a, cs->id[y]))
        before = core_ref(a, cs->id[x]) < core_ref(a, cs->id[y]);
      else before = cs->id[x] < cs->id[y];
      if (!before) break;
      slots[j + 1] = y;
    }
    slots[j + 1] = x;
  }
}

/* groups keyed by node (by_socket = 0) or socket (1) of full-free (filter_full) cores, cores sorted per group */
static void cores_by(const acc_t *a, const cores_t *cs, int filter_full, int by_socket, groups_t *g) {
  const ko_topo *t = a->t;
  int keys[N], nk = 0, nm[N];
  static __thread int members[N][N];
  for (int i = 0; i < cs->n; ++i) {
    if (filter_full && cs->n_cpus[i] != cpus_per_core(t)) continue;
    const int c0 = cs->cpus[i][0];
    const int key = by_socket ? t->socket[c0] : t->node[c0];
    int k = 0;
    while (k < nk && keys[k] != key) ++k;
    if (k == nk) { keys[nk] = key; nm[nk] = 0; ++nk; }
    members[k][nm[k]++] = i;
  }
  g->n = 0;
  int o = 0;
  for (int k = 0; k < nk; ++k) {
    sort_cores(a, cs, members[k], nm[k]);
    g->id[g->n] = keys[k];
    g->beg[g->n] = o;
    for (int m = 0; m < nm[k]; ++m) {
      const int s = members[k][m];
      int tmp[8];
      memcpy(tmp, cs->cpus[s], sizeof(int) * cs->n_cpus[s]);
      sort_ints(tmp, cs->n_cpus[s]);
      for (int q = 0; q < cs->n_cpus[s]; ++q) g->cpus[o++] = tmp[q];
    }
    g->len[g->n] = o - g->beg[g->n];
    ++g->n;
  }
}

/* stable insertion sort of the group order by a comparator on (a, g, i, j) */
typedef int (*grp_before)(const acc_t *a, const groups_t *g, const int *aux, int i, int j);
static void sort_groups(const acc_t *a, groups_t *g, const int *aux, grp_before before) {
  int ord[N];
  for (int i = 0; i < g->n; ++i) ord[i] = i;
  for (int i = 1; i < g->n; ++i) {
    const int x = ord[i];
    int j = i - 1;
    while (j >= 0 && before(a, g, aux, x, ord[j])) { ord[j + 1] = ord[j]; --j; }
    ord[j + 1] = x;
  }
  groups_t h = *g;
  for (int i = 0; i < g->n; ++i) {
    g->id[i] = h.id[ord[i]];
    g->beg[i] = h.beg[ord[i]];
    g->len[i] = h.len[ord[i]];
  }
}

/* freeCoresInNode: nodes by (len strategy, socket free strategy, node id) */
static int before_core_nodes(const acc_t *a, const groups_t *g, const int *socket_free, int i, int j) {
  int r = strat_cmp(a, g->len[i], g->len[j]);
  if (r) return r < 0;
  const int si = a->t->socket[g->cpus[g->beg[i]]], sj = a->t->socket[g->cpus[g->beg[j]]];
  r = strat_cmp(a, socket_free[si], socket_free[sj]);
  if (r) return r < 0;
  return g->id[i] < g->id[j];
}

static void free_cores_in_node(const acc_t *a, int filter_full, int filter_exclusive, groups_t *g) {
  cores_t cs;
  cs.n = 0;
  int socket_free[N];
  memset(socket_free, 0, sizeof socket_free);
  for (int c = 0; c < a->t->ncpus; ++c) {
    if (!a->alloc[c]) continue;
    if (filter_exclusive && excl_numa(a, c)) continue;
    const int s = core_slot(&cs, a->t->core[c]);
    cs.cpus[s][cs.n_cpus[s]++] = c;
    socket_free[a->t->socket[c]]++;
  }
  cores_by(a, &cs, filter_full, 0, g);
  sort_groups(a, g, socket_free, before_core_nodes);
}

static int before_len_id(const acc_t *a, const groups_t *g, const int *aux, int i, int j) {
  const int r = strat_cmp(a, g->len[i], g->len[j]);
  if (r) return r < 0;
  return g->id[i] < g->id[j];
}

static void free_cores_in_socket(const acc_t *a, int filter_full, groups_t *g) {
  cores_t cs;
  cs.n = 0;
  for (int c = 0; c < a->t->ncpus; ++c) {
    if (!a->alloc[c]) continue;
    const int s = core_slot(&cs, a->t->core[c]);
    cs.cpus[s][cs.n_cpus[s]++] = c;
  }
  cores_by(a, &cs, filter_full, 1, g);
  sort_groups(a, g, NULL, before_len_id);
}

/* extractCPU: the first CPU of each core, in list order */
static int extract(const acc_t *a, int *v, int n) {
  int seen[N], ns = 0, k = 0;
  for (int i = 0; i < n; ++i) {
    const int core = a->t->core[v[i]];
    if (has(seen, ns, core)) continue;
    seen[ns++] = core;
    v[k++] = v[i];
  }
  return k;
}

/* CPUs grouped by node (by_socket 0) or socket (1); sorted, refcount-sorted, extracted */
static void cpus_by(const acc_t *a, int by_socket, int filter_exclusive, groups_t *g, int *node_free, int *socket_free) {
  const ko_topo *t = a->t;
  int keys[N], nk = 0, nm[N];
  static __thread int members[N][N];
  for (int c = 0; c < t->ncpus; ++c) {
    if (!a->alloc[c]) continue;
    if (filter_exclusive && (by_socket ? excl_pcpu(a, c) : (excl_pcpu(a, c) || excl_numa(a, c)))) continue;
    const int key = by_socket ? t->socket[c] : t->node[c];
    int k = 0;
    while (k < nk && keys[k] != key) ++k;
    if (k == nk) { keys[nk] = key; nm[nk] = 0; ++nk; }
    members[k][nm[k]++] = c;
    if (node_free) node_free[t->node[c]]++;
    if (socket_free) socket_free[t->socket[c]]++;
  }
  g->n = 0;
  int o = 0;
  for (int k = 0; k < nk; ++k) {
    int *v = members[k];
    int n = nm[k];
    sort_ints(v, n);
    if (a->max_ref > 1) sort_by_ref(a, v, n);
    if (filter_exclusive) n = extract(a, v, n);
    g->id[g->n] = keys[k];
    g->beg[g->n] = o;
    for (int i = 0; i < n; ++i) g->cpus[o++] = v[i];
    g->len[g->n] = n;
    ++g->n;
  }
}

static int before_cpu_nodes(const acc_t *a, const groups_t *g, const int *aux, int i, int j) {
  const int *node_free = aux, *socket_free = aux + N;
  const int ci = g->cpus[g->beg[i]], cj = g->cpus[g->beg[j]];
  int r = strat_cmp(a, node_free[a->t->node[ci]], node_free[a->t->node[cj]]);
  if (r) return r < 0;
  r = strat_cmp(a, socket_free[a->t->socket[ci]], socket_free[a->t->socket[cj]]);
  if (r) return r < 0;
  return g->id[i] < g->id[j];
}

static void free_cpus_in_node(const acc_t *a, int filter_exclusive, groups_t *g) {
  int aux[2 * N];
  memset(aux, 0, sizeof aux);
  cpus_by(a, 0, filter_exclusive, g, aux, aux + N);
  sort_groups(a, g, aux, before_cpu_nodes);
}

static void free_cpus_in_socket(const acc_t *a, int filter_exclusive, groups_t *g) {
  cpus_by(a, 1, filter_exclusive, g, NULL, NULL);
  sort_groups(a, g, NULL, before_len_id);
}

/* freeCPUs: every free CPU, cores ordered by (socket colocation with the result desc, socket free
 * strategy, node free strategy, core free asc, socket id asc, refcount asc, core id asc) */
static int free_cpus(const acc_t *a, int filter_exclusive, int *out) {
  const ko_topo *t = a->t;
  cores_t cs;
  cs.n = 0;
  int node_free[N], socket_free[N], colo[N];
  memset(node_free, 0, sizeof node_free);
  memset(socket_free, 0, sizeof socket_free);
  for (int c = 0; c < t->ncpus; ++c) {
    if (!a->alloc[c]) continue;
    if (filter_exclusive && (excl_pcpu(a, c) || excl_numa(a, c))) continue;
    const int s = core_slot(&cs, t->core[c]);
    cs.cpus[s][cs.n_cpus[s]++] = c;
    node_free[t->node[c]]++;
    socket_free[t->socket[c]]++;
  }
  memset(colo, 0, sizeof colo);
  for (int c = 0; c < t->ncpus; ++c)
    if (a->result[c]) colo[t->socket[c]]++;
  int ord[N];
  for (int i = 0; i < cs.n; ++i) ord[i] = i;
  for (int i = 1; i < cs.n; ++i) {
    const int x = ord[i];
    int j = i - 1;
    for (; j >= 0; --j) {
      const int y = ord[j];
      const int cx = cs.cpus[x][0], cy = cs.cpus[y][0];
      const int sx = t->socket[cx], sy = t->socket[cy], nx = t->node[cx], ny = t->node[cy];
      int before, r;
      if (colo[sx] != colo[sy]) before = colo[sx] > colo[sy];
      else if ((r = strat_cmp(a, socket_free[sx], socket_free[sy]))) before = r < 0;
      else if ((r = strat_cmp(a, node_free[nx], node_free[ny]))) before = r < 0;
      else if (cs.n_cpus[x] != cs.n_cpus[y]) before = cs.n_cpus[x] < cs.n_cpus[y];
      else if (sx != sy) before = sx < sy;
      else if (a->max_ref > 1 && core_ref(a, cs.id[x]) != core_ref(a, cs.id[y]))
        before = core_ref(a, cs.id[x]) < core_ref(a, cs.id[y]);
      else before = cs.id[x] < cs.id[y];
      if (!before) break;
      ord[j + 1] = y;
    }
    ord[j + 1] = x;
  }
  int k = 0;
  for (int i = 0; i < cs.n; ++i) {
    const int s = ord[i];
    int tmp[8];
    memcpy(tmp, cs.cpus[s], sizeof(int) * cs.n_cpus[s]);
    sort_ints(tmp, cs.n_cpus[s]);
    if (a->max_ref > 1) sort_by_ref(a, tmp, cs.n_cpus[s]);
    for (int q = 0; q < cs.n_cpus[s]; ++q) out[k++] = tmp[q];
  }
  return k;
}

/* spreadCPUs: passes that take the first not-yet-seen core's CPU */
static int spread(const acc_t *a, int *v, int n) {
  if (n <= cpus_per_core(a->t)) return n;
  int prep[N], np = n, out = 0;
  memcpy(prep, v, sizeof(int) * n);
  while (np > 0) {
    int res[N], nr = 0, seen[N], ns = 0;
    for (int i = 0; i < np; ++i) {
      const int core = a->t->core[prep[i]];
      if (has(seen, ns, core)) { res[nr++] = prep[i]; continue; }
      v[out++] = prep[i];
      seen[ns++] = core;
    }
    memcpy(prep, res, sizeof(int) * nr);
    np = nr;
  }
  return out;
}

static void acc_init(acc_t *a, const ko_topo *t, int max_ref, const uint8_t *avail, const int32_t *refcount,
                     const int8_t *excl, int needed, int excl_policy, int strategy) {
  memset(a, 0, sizeof *a);
  a->t = t;
  a->max_ref = max_ref;
  for (int c = 0; c < t->ncpus; ++c) {
    if (excl && excl[c] == KO_EXCL_PCPU && !has(a->excl_cores, a->n_excl_cores, t->core[c]))
      a->excl_cores[a->n_excl_cores++] = t->core[c];
    else if (excl && excl[c] == KO_EXCL_NUMA && !has(a->excl_nodes, a->n_excl_nodes, t->node[c]))
      a->excl_nodes[a->n_excl_nodes++] = t->node[c];
    a->alloc[c] = avail[c] ? 1 : 0;
    a->ref[c] = (max_ref > 1 && refcount) ? refcount[c] : 0;
  }
  a->exclusive = excl_policy == KO_EXCL_PCPU || excl_policy == KO_EXCL_NUMA;
  a->excl_policy = excl_policy;
  a->strategy = strategy;
  a->needed = needed;
}

int ko_take_cpus(const ko_topo *t, int max_ref, const uint8_t *avail, const int32_t *refcount, const int8_t *excl,
                 int needed, int bind, int excl_policy, int strategy, uint8_t *out) {
  static __thread acc_t a;
  static __thread groups_t g;
  int list[N];
  acc_init(&a, t, max_ref, avail, refcount, excl, needed, excl_policy, strategy);
  memset(out, 0, (size_t)t->ncpus);
  if (satisfied(&a)) return 0;
  if (a.needed > n_alloc(&a)) return -1;
  const int full = bind == KO_BIND_FULL_PCPUS;
  const int cpc = cpus_per_core(t);
  if (full || cpc == 1) {
    if (a.needed <= cpus_per_node(t)) {
      for (int fe = 1; fe >= 0; --fe) {
        free_cores_in_node(&a, 1, fe, &g);
        for (int i = 0; i < g.n; ++i)
          if (g.len[i] >= a.needed) {
            take(&a, g.cpus + g.beg[i], a.needed);
            goto done;
          }
      }
    }
    if (a.needed <= cpus_per_socket(t)) {
      free_cores_in_socket(&a, 1, &g);
      for (int i = 0; i < g.n; ++i)
        if (g.len[i] >= a.needed) {
          take(&a, g.cpus + g.beg[i], a.needed);
          goto done;
        }
    }
    free_cores_in_socket(&a, 1, &g);
    /* sort.Slice by len desc (stable for <= 12 sockets) */
    int ord[N], nu = 0, uns[N];
    for (int i = 0; i < g.n; ++i) ord[i] = i;
    for (int i = 1; i < g.n; ++i) {
      const int x = ord[i];
      int j = i - 1;
      while (j >= 0 && g.len[x] > g.len[ord[j]]) { ord[j + 1] = ord[j]; --j; }
      ord[j + 1] = x;
    }
    for (int i = 0; i < g.n; ++i) {
      const int k = ord[i];
      if (!needs(&a, g.len[k])) {
        uns[nu++] = k;
      } else {
        take(&a, g.cpus + g.beg[k], g.len[k]);
        if (satisfied(&a)) goto done;
      }
    }
    if (needs(&a, cpc)) {
      for (int i = 1; i < nu; ++i) {  /* sort.Slice by len asc (stable) */
        const int x = uns[i];
        int j = i - 1;
        while (j >= 0 && g.len[x] < g.len[uns[j]]) { uns[j + 1] = uns[j]; --j; }
        uns[j + 1] = x;
      }
      for (int i = 0; i < nu; ++i) {
        const int k = uns[i];
        for (int q = 0; q < g.len[k]; q += cpc) {
          take(&a, g.cpus + g.beg[k] + q, cpc);
          if (satisfied(&a)) goto done;
          if (!needs(&a, cpc)) break;
        }
      }
    }
  }
  if (!full) {
    if (a.needed <= cpus_per_node(t)) {
      for (int fe = 1; fe >= 0; --fe) {
        free_cpus_in_node(&a, fe, &g);
        for (int i = 0; i < g.n; ++i)
          if (g.len[i] >= a.needed) {
            memcpy(list, g.cpus + g.beg[i], sizeof(int) * g.len[i]);
            spread(&a, list, g.len[i]);
            take(&a, list, a.needed);
            goto done;
          }
      }
    }
    if (a.needed <= cpus_per_socket(t)) {
      for (int fe = 1; fe >= 0; --fe) {
        free_cpus_in_socket(&a, fe, &g);
        for (int i = 0; i < g.n; ++i)
          if (g.len[i] >= a.needed) {
            memcpy(list, g.cpus + g.beg[i], sizeof(int) * g.len[i]);
            spread(&a, list, g.len[i]);
            take(&a, list, a.needed);
            goto done;
          }
      }
    }
  }
  for (int fe = 1; fe >= 0; --fe) {
    int n = free_cpus(&a, fe, list);
    n = spread(&a, list, n);
    for (int i = 0; i < n; ++i) {
      if (needs(&a, 1)) take(&a, &list[i], 1);
      if (satisfied(&a)) goto done;
    }
  }
  return -1;
done:
  memcpy(out, a.result, (size_t)t->ncpus);
  return 0;
}

int ko_spread_order(const ko_topo *t, int strategy, int *order) {
  static __thread acc_t a;
  uint8_t avail[N];
  memset(avail, 1, sizeof avail);
  acc_init(&a, t, 1, avail, NULL, NULL, 0, KO_EXCL_NONE, strategy);
  const int n = free_cpus(&a, 0, order);
  return spread(&a, order, n);
}

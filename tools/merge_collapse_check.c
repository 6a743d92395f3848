// Exhaustive check (a proof over the finite case space): is the topology-manager merge over L identical
// DeviceShare lists (one per requested device resource, topology_hint.go) the merge over one of them?  K <= 2
// NUMA nodes (the only case with device hints), every NodeNUMAResource list shape (absent / {nil,false} /
// any hint subset with any min size), every weak order of the three mask scores, every DeviceShare list shape
// over NUMA ids {0}, {1}, {0,1}, L = 2..4, all three policies; both merges are the oracle's ko_topology_merge
// (pinned by the reference's policy_test.go tables).  Build: see tests/test_merge_collapse.py.
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
int ko_topology_merge(int policy, int K, int nlists, const int *lens, const uint32_t *masks, const int *prefs,
                      const int64_t *scores, uint32_t *affinity, int *preferred);
typedef struct { int n; uint32_t m[4]; int p[4]; int64_t s[4]; } L;
static int run(int pol, int K, L *ls, int nl, uint32_t *aff, int *pref) {
  int lens[8]; uint32_t m[64]; int p[64]; int64_t s[64]; int o = 0;
  for (int l = 0; l < nl; l++) { lens[l] = ls[l].n; for (int i = 0; i < ls[l].n; i++, o++) { m[o] = ls[l].m[i]; p[o] = ls[l].p[i]; s[o] = ls[l].s[i]; } }
  return ko_topology_merge(pol, K, nl, lens, m, p, s, aff, pref);
}
int main(void) {
  long cases = 0, bad = 0;
  for (int K = 1; K <= 2; K++) {
    const uint32_t masks[3] = {1, 2, 3};
    const int nm = K == 1 ? 1 : 3;
    // NUMA list options: -1 absent, 0 nil-false, else subset bits (1..2^nm-1) with min_size
    int nopt = 0; int ob[40], oms[40];
    ob[nopt] = -1; oms[nopt++] = 0; ob[nopt] = 0; oms[nopt++] = 0;
    for (int b = 1; b < (1 << nm); b++) for (int ms = 1; ms <= K; ms++) {
      int minpc = 9; for (int i = 0; i < nm; i++) if ((b >> i) & 1) { int pc = __builtin_popcount(masks[i]); if (pc < minpc) minpc = pc; }
      if (ms > minpc) continue; ob[nopt] = b; oms[nopt++] = ms; }
    // DS options over id sets
    for (int pol = 1; pol <= 3; pol++)
    for (int sc = 0; sc < (nm == 3 ? 27 : 3); sc++) {
      int64_t hs[3] = {sc % 3, (sc / 3) % 3, sc / 9};
      for (int a = 0; a < nopt; a++) for (int b = 0; b < nopt; b++) {
        L base[8]; int nb = 0;
        int opts[2] = {a, b};
        for (int r = 0; r < 2; r++) {
          int o = opts[r]; if (ob[o] == -1) continue;
          L l = {0};
          if (ob[o] == 0) { l.n = 1; l.m[0] = 0; l.p[0] = 0; l.s[0] = 0; }
          else for (int i = 0; i < nm; i++) if ((ob[o] >> i) & 1) { l.m[l.n] = masks[i]; l.p[l.n] = __builtin_popcount(masks[i]) == oms[o]; l.s[l.n++] = hs[i]; }
          base[nb++] = l;
        }
        if (nb == 0) { L l = {1, {0}, {1}, {0}}; base[nb++] = l; }
        // DS masks: ids {0,1} -> [1,2,3] (K==2 only), {0} -> [1], {1} -> [2] (K==2)
        for (int idset = 0; idset < (K == 2 ? 3 : 1); idset++) {
          uint32_t dm[3]; int nd;
          if (idset == 0) { dm[0] = 1; nd = 1; } else if (idset == 1) { dm[0] = 2; nd = 1; } else { dm[0] = 1; dm[1] = 2; dm[2] = 3; nd = 3; }
          for (int okb = 0; okb < (1 << nd); okb++) for (int minaff = 1; minaff <= (nd == 3 ? 2 : 1); minaff++) {
            L d = {0};
            if (okb == 0) { d.n = 1; d.m[0] = 0; d.p[0] = 0; }
            else for (int i = 0; i < nd; i++) if ((okb >> i) & 1) { d.m[d.n] = dm[i]; d.p[d.n] = __builtin_popcount(dm[i]) == minaff; d.s[d.n++] = 0; }
            L one[8]; memcpy(one, base, sizeof(L) * nb); one[nb] = d;
            uint32_t a1; int p1; int r1 = run(pol, K, one, nb + 1, &a1, &p1);
            for (int Lc = 2; Lc <= 4; Lc++) {
              L many[8]; memcpy(many, base, sizeof(L) * nb);
              for (int q = 0; q < Lc; q++) many[nb + q] = d;
              uint32_t a2; int p2; int r2 = run(pol, K, many, nb + Lc, &a2, &p2);
              cases++;
              if (r1 != r2 || a1 != a2 || p1 != p2) { if (bad < 5) printf("mismatch K=%d pol=%d a=%d b=%d ids=%d ok=%d minaff=%d L=%d: %d/%x/%d vs %d/%x/%d\n", K, pol, a, b, idset, okb, minaff, Lc, r1, a1, p1, r2, a2, p2); bad++; }
            }
          }
        }
      }
    }
  }
  printf("cases %ld mismatches %ld\n", cases, bad);
  return 0;
}

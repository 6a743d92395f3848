import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0, 'tests')
import numpy as np
from helpers import *
from koordinator_amd import runtime as rt
from oracle.oracle import Oracle
rng = np.random.Generator(np.random.PCG64(13))
nodes = stress_nodes(1500, rng, tight=True)
pods = stress_pods(1200, rng, n_quotas=24)
quotas = nested_quotas(pods, rng, 24)
for prof in (profile(quota=True, prod_usage=True), profile(quota=True, check_parent=True, candidates=3), profile(quota=False, prod_usage=True), profile(quota=True)):
    cfg = prof.to_ks_config()
    for b in (1, 64):
        cfg.batch_pods = b
        ev = rt.Evaluator(cfg, nodes.copy(), quotas.copy())
        g = ev.schedule(pods)
        o = Oracle(cfg, nodes.copy(), quotas.copy())
        w = o.schedule(pods)
        bad = np.nonzero((g['node'] != w['node']) | (g['status'] != w['status']))[0]
        print('quota', cfg.quota.enable, 'parent', cfg.quota.enable_check_parent_quota, 'prod', cfg.loadaware.score_according_prod_usage, 'batch', b, 'ndiff', len(bad), bad[:5], ev.stats())
# prefix check
cfg = profile(quota=True, prod_usage=True).to_ks_config()
for k in (1, 2, 3, 4, 5):
    ev = rt.Evaluator(cfg, nodes.copy(), quotas.copy()); g = ev.schedule(pods.rows(range(k)))
    o = Oracle(cfg, nodes.copy(), quotas.copy()); w = o.schedule(pods.rows(range(k)))
    sg, so = ev.read_nodes().as_dict(), o.read_nodes().as_dict()
    diffs = {kk: np.nonzero(np.asarray(sg[kk]) != np.asarray(so[kk]))[-1][:5].tolist() for kk in so if not np.array_equal(sg[kk], so[kk])}
    print(k, g['node'], w['node'], diffs, (ev.read_quota_used() != o.read_quota_used()).sum())
    one = pods.rows([k])
    rg, sg2, tg = ev.eval_pod(one); ro, so2, to = o.eval_pod(one)
    print('  eval next pod diff nodes:', np.nonzero((rg != ro) | (tg != to))[0][:10], 'gpu best', tg.max(), tg.argmax(), 'orc best', to.max(), to.argmax())

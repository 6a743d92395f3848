import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sys; sys.path.insert(0,'tests')
import numpy as np
from helpers import *
from koordinator_amd import runtime as rt
rng=np.random.Generator(np.random.PCG64(7))
nodes=stress_nodes(777,rng); pods=stress_pods(64,rng)
ev=rt.Evaluator(profile().to_ks_config(), nodes)
try:
    print(ev.schedule(pods.rows(range(10))))
except Exception as e: print("sched", e)
try:
    print(ev.eval_pod(pods.rows([0]))[2][:10])
except Exception as e: print("eval", e)

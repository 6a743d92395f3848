"""CPU oracle for koord-scheduler's per-pod sweep — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / baseline timer.  The
product (``libkoordgpu.so`` and ``koordinator_amd``) never imports it.

* ``koord_oracle.c``   scalar C restatement of the reduced-form sweep and the
  reference's 16-worker Parallelizer (see the file header for file:line refs).
* ``loadaware_ref.py`` pure-Python restatement of the LoadAware plugin at object
  level (Filter/Score/EstimatePod/EstimateNode), used on the golden vectors.
* ``quota_runtime_ref.py`` ElasticQuota RefreshRuntime (request aggregation + water-filling).

Parity status: pinned by the reference's own test tables transcribed into
``tests/golden/`` (LoadAware TestFilterUsage / TestScore / estimator tests,
ElasticQuota TestPlugin_PreFilter*, runtime calculator and group-quota-manager runtime tests).  NodeResourcesFit and the sweep driver live
in upstream kube-scheduler (not on disk): those parts are parity-unpinned.
"""

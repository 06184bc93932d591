"""CPU oracle for the MOPO model-rollout + SAC-update hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``mopo_amd/`` imports this package: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may use it, and only as the checker / timed CPU baseline, never as the thing
measured or shipped.

Every function restates the reference algorithm in numpy and cites the
reference file:line it follows (paths are relative to the reference repo
xionghuichen/mopo).  Pinning:

* ``fake_env``, ``static_fns`` and ``replay_pool`` are pinned against golden
  vectors produced by executing the reference's own ``FakeEnv.step``,
  ``mopo/static/*.py`` and ``FlexibleReplayPool`` (see
  ``tests/golden/make_golden.py``).
* ``bnn`` (TF1 graph) and ``sac`` (TF1 graph) cannot run here (TensorFlow 1.14
  is absent); they are restatements whose fixtures are labelled
  "restatement-pinned".  ``sac`` is additionally cross-checked against torch
  autograd in ``tests/test_oracle.py``.
* ``rng`` follows numpy's legacy ``RandomState`` (MT19937) and is checked
  bit-exact against numpy itself.
"""

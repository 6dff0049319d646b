"""CPU oracle for the MARL-Maze hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this package, and only as the checker (or as the timed
CPU baseline).  The product package ``marl-maze_amd/marlmaze`` never imports it
and fails loudly when its HIP library is missing.

Contents (each restates the reference, rhuangr/MARL-Maze @ 2024-10-08):

* ``maze_oracle.c`` / :mod:`oracle.env` -- the environment (maze generation with
  CPython's MT19937, ``Maze.step``, ``Agent.get_observations``), plain C.
* :mod:`oracle.ppo` -- GAE (numpy fp32 restatement of ``PPO.get_GAEs``), the
  Actor/Critic networks and the PPO update in torch fp32 on the CPU, and a
  single-maze ``train()`` port used as the CPU baseline.

Parity pinning: both are checked against the golden vectors in ``tests/golden``
that ``tests/golden/make_golden.py`` captured by importing the reference.
"""

"""ORACLE — test infrastructure, NOT product code.

A CPU restatement (numpy, fp32 / fp64 / integer) of the reference's v18
embedding-RAG hot path, used only as the checker:

* ``tests/``                      — parity tests compare the HIP path with it,
* ``__graft_entry__.smoke()``     — one small invocation checked against it,
* ``bench.py`` (``cpu_baseline``) — timed on the host cores as the "port" baseline.

Nothing in ``rag-snvbert_amd/`` imports, calls or links anything here; the
product path fails loudly when the HIP library is missing instead of falling
back to this code.

Pinning: every function cites the reference ``file:line`` it restates, and
``tests/test_oracle_golden.py`` checks it against fixtures produced by RUNNING
the reference itself (``tests/golden/make_golden.py``: the real
``src/model`` modules, and the reference's own dataset/retrieval functions
executed from their source text).
"""

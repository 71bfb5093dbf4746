"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of FL_PyTorch's simulated-uplink hot path, used as the *checker* for the
MI355X product in ``flpytorch_amd/``.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this package; the product never does (and
fails loudly if its HIP library is missing instead of falling back to anything here).

Pinned against the real reference: ``tests/golden/`` holds fixtures produced by importing
``/root/reference/fl_pytorch`` in the development container (``tests/golden/make_golden.py``)
— codec outputs, numpy-stream draws and ``run.py`` round captures.  ``tests/test_oracle_golden.py``
checks this package against every one of them.

Modules
-------
- ``oracle.rng``    numpy-legacy MT19937 stream (C, ``oracle/mt19937_legacy.c``) via ctypes.
- ``oracle.codecs`` op-for-op numpy restatement of ``Compressor`` (compressors.py:22-494) and
                    of the ``serverGradient`` reduction (algorithms.py:1748-1770, 1810-1832).
"""

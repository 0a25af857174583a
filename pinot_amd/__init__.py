"""pinot_amd -- MI355X-native server-side segment execution path for Apache Pinot.

The product is ``libpinot_hip.so`` (C-ABI, ``include/pinot_hip.h``): HBM-pinned segments and
hand-written gfx950 HIP kernels for the filter -> aggregation / group-by path.  This package is
the Python host binding (ctypes) used by tests and the benchmark, mirroring the reference's
QueryContext / ServerQueryExecutor interface.
"""

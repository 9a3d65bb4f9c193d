"""MI355X-native event-binning engine for ESS live data reduction.

Drop-in replacement for the detector-view and monitor-histogram hot path of
scipp/esslivedata: ev44 events -> pixel/screen projection -> TOA binning ->
cumulative/current histograms, computed by hand-written CDNA4 HIP kernels
behind a C ABI (``include/lde.h``) and the reference's own ``Accumulator`` /
``Workflow`` plugin protocols.
"""

__version__ = '0.1.0'

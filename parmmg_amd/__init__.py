"""parmmg_amd — MI355X-native replacement of ParMmg's old->new mesh transfer
step (PMMG_interpMetricsAndFields, reference src/interpmesh_pmmg.c:663-741).

The product is the HIP module ``libpmmg_hip.so`` behind the C-ABI of
``include/parmmg_hip.h`` plus the C host layer ``libpmmg_host.so``; this
package only builds and binds them (``build``, ``_native``, ``transfer``) and
provides the synthetic workloads (``synth``, ``configs``).
"""
from .transfer import TransferContext, device_count, interp_metrics_and_fields  # noqa: F401

__all__ = ["TransferContext", "device_count", "interp_metrics_and_fields"]

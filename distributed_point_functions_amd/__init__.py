"""MI355X-native DPF tree expansion + dense-PIR scan (gfx950 HIP kernels).

A from-scratch implementation of the hot path of Google's incremental
Distributed Point Functions library (d346uvcdd/distributed_point_functions)
behind the reference's API: `DistributedPointFunction`
(CreateIncremental / GenerateKeys / CreateEvaluationContext / EvaluateNext /
EvaluateUntil / EvaluateAt / EvaluateAndApply), `DistributedComparisonFunction`
(GenerateKeys / Evaluate / BatchEvaluate) and `DenseDpfPirServer`
(HandleRequest).  All evaluation runs in hand-written HIP kernels reached
through the C ABI of include/dpf_amd.h; there is no CPU evaluation path.
"""
from . import value_types, wire  # noqa: F401
from .value_types import (Integer, IntModN, Tuple, ValueType,  # noqa: F401
                          XorWrapper)

__all__ = ["value_types", "wire", "Integer", "IntModN", "Tuple", "ValueType",
           "XorWrapper"]


def __getattr__(name):
    import importlib
    if name in ("DistributedPointFunction", "DpfParameters", "DpfKey",
                "EvaluationContext"):
        return getattr(importlib.import_module(__name__ + ".dpf"), name)
    if name in ("DistributedComparisonFunction", "DcfParameters", "DcfKey"):
        return getattr(importlib.import_module(__name__ + ".dcf"), name)
    if name in ("DenseDpfPirDatabase", "DenseDpfPirServer", "PirConfig"):
        return getattr(importlib.import_module(__name__ + ".pir"), name)
    if name in ("kernels", "dpf", "dcf", "pir"):
        return importlib.import_module(__name__ + "." + name)
    raise AttributeError(name)

"""hyperopt_amd -- MI355X-native TPE suggestion engine behind hyperopt's API.

The numeric hot path of ``tpe.suggest`` (split, Parzen fit, candidate draws,
GMM/LGMM/categorical lpdf, EI argmax) runs as hand-written gfx950 HIP kernels
in ``libtpe_engine.so`` (C ABI: include/tpe_engine.h).
"""
__version__ = '0.1.0'

"""Drop-in aggregation plug-in: codecs + server reduction on MI355X.

``install(compressors_module, algorithms_module)`` rebinds the reference's
``utils.compressors.initCompressor`` / ``Compressor`` and the ``serverGradient`` of the algorithm
classes whose reduction is the shared sequential fold (algorithms.py:1753-1768), so
``fl_pytorch/run.py`` runs unchanged on top of libflcodec.
"""
from .compressors import (Compressor, CompressorType, initCompressor, stream_choice, stream_rand,  # noqa: F401
                          stream_random, stream_randint31)
from .fused import PayloadReducer, UplinkReducer, select_row_flags  # noqa: F401
from .mixed import MixedUplink  # noqa: F401
from .shift import dianaStep, ef21Step, marinaStep  # noqa: F401
from .reduce import (make_server_gradient_frecon, reduce_client_models, reduce_rows,  # noqa: F401
                     serverGradientCOFIG, serverGradientDIANA, serverGradientGradSkip, serverGradientMaster,
                     serverGradientPlain)

# Algorithm classes whose serverGradient is exactly the shared fold, and what follows it.
PLAIN_FOLD = ("FedAvg", "FedProx",                  # return gs            (1810-1832, 1886-1908,
              "MarinaAlgorithm", "MarinaAlgorithmPP", "SCAFFOLD")  #        545-563, 699-717, 792-814)
MASTER_FOLD = ("DCGD", "EF21", "EF21PP")            # master compressor    (1748-1770, 1521-1546, 1654-1679)
SHIFTED_FOLD = {"DIANA": serverGradientDIANA,       # H['m'] = gs; h + gs  (1395-1421)
                "COFIG": serverGradientCOFIG,       # u + h_prev, updates  (1273-1307)
                "GradSkip": serverGradientGradSkip}  # fold of x_i - h_i gamma / p, delta_x   (951-998)
# FRECON (1124-1176) folds the clients' q_i as well and takes lambda from the reference module's
# experiment-option helpers: its serverGradient is built per installed module.


def install(compressors_module, algorithms_module=None):
    """Rebind the reference's codec factory and reducers to the MI355X implementations.

    Returns a callable that restores the originals."""
    saved = [(compressors_module, "initCompressor", compressors_module.initCompressor),
             (compressors_module, "Compressor", compressors_module.Compressor)]
    compressors_module.initCompressor = initCompressor
    compressors_module.Compressor = Compressor
    if algorithms_module is not None:
        for name, fn in ([(n, serverGradientPlain) for n in PLAIN_FOLD] + [(n, serverGradientMaster) for n in MASTER_FOLD]
                         + list(SHIFTED_FOLD.items())):
            cls = getattr(algorithms_module, name, None)
            if cls is None:
                continue
            saved.append((cls, "serverGradient", cls.__dict__["serverGradient"]))
            cls.serverGradient = staticmethod(fn)
        frecon = getattr(algorithms_module, "FRECON", None)
        if frecon is not None:
            saved.append((frecon, "serverGradient", frecon.__dict__["serverGradient"]))
            frecon.serverGradient = staticmethod(make_server_gradient_frecon(algorithms_module))

    def restore():
        for obj, attr, val in reversed(saved):
            setattr(obj, attr, val)
    return restore

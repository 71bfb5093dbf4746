"""Client steps of the compressed algorithms on the shift codecs.

Each helper is the torch expression of the reference's ``localGradientEvaluation`` after the local
gradient is known, executed as ONE ``flc_encode_shift`` call (``Compressor.compressShift``): the
compressed difference is never materialised for the elementwise codecs, and the shift / estimator
update is written in the same pass.  Results are bit-identical to the reference's expressions
(tests/test_gpu_shift.py).  Wire statistics advance exactly as the reference's compressVector call.
"""


def dianaStep(compressor, grad_cur, h, alpha, in_place=False):
    """DIANA (algorithms.py:1383-1391), also FRECON's / COFIG's u_i (1104-1110, 1265-1269):
    ``m_i = C(grad - h); h = h + alpha * m_i``.  Returns ``(m_i, h_new)``; ``in_place`` writes
    h_new over ``h`` (the reference rebinds a new tensor: keep the default unless h is owned)."""
    return compressor.compressShift(grad_cur, h, alpha=alpha, shift=h, shift_out=h if in_place else None)


def ef21Step(compressor, grad_cur, g_prev, in_place=False):
    """EF21 (algorithms.py:1506-1517): ``g_next = g_prev + C(grad - g_prev) * mult`` with
    ``mult = 1 / (1 + w)`` for an unbiased (non-contraction) codec, else 1."""
    mult = 1.0
    if not compressor.isContractionCompressor():
        mult = 1.0 / (1.0 + compressor.getW())
    msg, _ = compressor.compressShift(grad_cur, g_prev, scale=mult, base=g_prev, out=g_prev if in_place else None)
    return msg


def marinaStep(compressor, grad_cur, grad_prev, g_prev):
    """MARINA / PP-MARINA (algorithms.py:537, 691): ``g_next = g_prev + C(grad_cur - grad_prev)``."""
    msg, _ = compressor.compressShift(grad_cur, grad_prev, base=g_prev)
    return msg

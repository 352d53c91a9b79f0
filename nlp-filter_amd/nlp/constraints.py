"""Constraint plug-ins -- kingdwd/nlp-filter nlp/constraints.py (signature kept;
on the GPU path as constraint index pairs of the bordered GN step)."""


def equality_constaint(x, params=None):
    """x[0] - x[1] (nlp/constraints.py:4-5; the reference's spelling is kept)"""
    return x[0] - x[1]

"""MI355X-native drop-in for kingdwd/nlp-filter's ``nlp`` package.

``nlp.nlp``            problem builder + solve facade (Gauss-Newton on libmhe.so)
``nlp.collocation``    Chebyshev pseudospectral constants
``nlp.dynamics`` / ``nlp.measurements`` / ``nlp.cost_functions`` / ``nlp.constraints``
                       plug-ins with the reference signatures
"""

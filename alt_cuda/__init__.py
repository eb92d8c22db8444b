"""Drop-in package for the reference's ``alt_cuda`` (alt_cuda/__init__.py is empty there).

``from alt_cuda.fw import FW`` (preprocess.py:17) resolves to the MI355X engine.
"""

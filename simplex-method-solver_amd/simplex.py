"""Drop-in replacement for jqnfxa/Simplex-Method-Solver's ``src/simplex.py``.

Put this directory on ``sys.path`` (or copy this file next to ``main.py``) and the reference UI's
imports -- ``from simplex import SimplexMethod, Error`` (main.py:13) and
``from simplex import Info`` (table_widget.py:7) -- resolve to the MI355X engine unchanged.
"""
from simplex_mi355x.engine import Error, Info, SimplexMethod

__all__ = ["SimplexMethod", "Info", "Error"]

"""ORACLE — test infrastructure only (CPU restatement of the reference path).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The product package ``zipvoice_amd`` never imports this package.
"""

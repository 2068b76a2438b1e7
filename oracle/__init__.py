"""ORACLE package — CPU restatements of the reference hot path. TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
Never imported by the product package `zonos_vibes_amd`.
"""

"""CPU oracle of the reference hot path -- test infrastructure only.

Importable solely from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  See DESIGN.md "Oracle" for provenance and pinning.
"""

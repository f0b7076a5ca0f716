"""Test-infrastructure oracle (CPU restatement of the reference hot path).

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  See rcan_oracle.py for the reference file:line map.
"""

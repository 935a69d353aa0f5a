"""ORACLE -- test infrastructure only.

CPU restatement of the reference's clip-embedding + one-shot matching path, pinned
against golden vectors captured from the reference itself (tests/golden/).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker / CPU baseline.  The product package never does.
"""

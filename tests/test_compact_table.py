"""Round-6 design check: an exact compact
byU16 hash table (h % S slots holding a tag + the 13-bit position, plus an
'evicted key' bitmap that sends a block back to the dense 16 KiB table when a
lookup would need an overwritten entry) would fit more encoder blocks per CU,
but the parse's own table traffic -- logged by a Python restatement of the
parse that is checked sequence-for-sequence against the oracle -- overflows it
in most bit-shuffled G1 / E = 3 blocks.  Full run: profiles/r06/compact_table_sim.txt
(python tests/compact_table_sim.py)."""
import numpy as np

from tests.compact_table_sim import blocks, lz4_log, o, oracle_seqs, replay


def test_compact_table_needs_the_dense_fallback_in_most_blocks():
    for name, arr, E in [("G1", o.gen_g1(1 << 18), 2), ("E3", o.gen_g1(1 << 18).view(np.uint8)[: (1 << 19) // 3 * 3], 3)]:
        exact = 0
        for b in blocks(arr, E, 6):
            log, seqs = lz4_log(b)
            assert seqs == oracle_seqs(o.lz4_compress_block(np.frombuffer(b, np.uint8)).tobytes())
            exact += replay(log, 4096)[0]
        assert exact <= 3, (name, exact)  # at least half the blocks would re-parse densely

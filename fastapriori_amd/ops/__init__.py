"""Mining primitives: HIP kernels for device tensors, C++ reference for CPU tensors."""
from .primitives import (apriori_gen_device, bitmap_geometry, build_bitmaps, compress, compress_rows, count_candidates, f1_exact, f1_sketch, histogram, sketch_estimate,  # noqa: F401
                         pair_counts_gram, count_level, trim_rows, pair_counts_horizontal, recommend, row_hash, txn_freq_count)

// mm_n12.hip — the kernels and host drivers of padded size N = 4096
// (log2 N = 12), in their own translation unit (mm_impl.hpp).
#include "mm_impl.hpp"

MM_SIZE_ENTRIES(12)

// mm_n06.hip — the kernels and host drivers of padded size N = 64
// (log2 N = 6), in their own translation unit (mm_impl.hpp).
#include "mm_impl.hpp"

MM_SIZE_ENTRIES(6)

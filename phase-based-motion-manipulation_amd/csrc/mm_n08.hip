// mm_n08.hip — the kernels and host drivers of padded size N = 256
// (log2 N = 8), in their own translation unit (mm_impl.hpp).
#include "mm_impl.hpp"

MM_SIZE_ENTRIES(8)

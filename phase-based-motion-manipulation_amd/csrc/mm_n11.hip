// mm_n11.hip — the kernels and host drivers of padded size N = 2048
// (log2 N = 11), in their own translation unit (mm_impl.hpp).
#include "mm_impl.hpp"

MM_SIZE_ENTRIES(11)

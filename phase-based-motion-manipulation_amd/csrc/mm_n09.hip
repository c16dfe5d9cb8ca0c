// mm_n09.hip — the kernels and host drivers of padded size N = 512
// (log2 N = 9), in their own translation unit (mm_impl.hpp).
#include "mm_impl.hpp"

MM_SIZE_ENTRIES(9)

// mm_n10.hip — the kernels and host drivers of padded size N = 1024
// (log2 N = 10), in their own translation unit (mm_impl.hpp).
#include "mm_impl.hpp"

MM_SIZE_ENTRIES(10)

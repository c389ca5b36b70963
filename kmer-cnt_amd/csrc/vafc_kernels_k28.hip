// vafc_kernels_k28.hip -- instantiates the counting kernels for k = 28, 29, 30, 31.
#include "vafc_scan.h"

hipError_t vc_launch_k28(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<28>(A, grid, grid_long, st);
}
hipError_t vc_setup_k28(int lds) { return setup_k<28>(lds); }

hipError_t vc_launch_k29(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<29>(A, grid, grid_long, st);
}
hipError_t vc_setup_k29(int lds) { return setup_k<29>(lds); }

hipError_t vc_launch_k30(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<30>(A, grid, grid_long, st);
}
hipError_t vc_setup_k30(int lds) { return setup_k<30>(lds); }

hipError_t vc_launch_k31(const VcKernelArgs *A, int grid, int grid_long, hipStream_t st)
{
	return launch_k<31>(A, grid, grid_long, st);
}
hipError_t vc_setup_k31(int lds) { return setup_k<31>(lds); }


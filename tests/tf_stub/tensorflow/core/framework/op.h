#pragma once
#include "op_kernel.h"

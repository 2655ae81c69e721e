#pragma once
#include "shim_headers.h"

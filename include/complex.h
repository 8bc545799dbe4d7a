/* forwarding header: the ns-nnsp API is declared in nnsp_api.h */
#include "nnsp_api.h"

/* include/refcompat/Vertex.h — forwards the reference's CG_Project/Vertex.h to the MI355X drop-in, so a host
 * whose sources include "Vertex.h" compiles unchanged when this directory replaces the reference's
 * headers (see include/raytracert_dropin.hpp and INTEGRATION.md). */
#pragma once
#include "../raytracert_dropin.hpp"

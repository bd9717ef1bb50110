// all.hpp -- every protocol with device transition functions.
#pragma once
#include "pingpong.hpp"
#include "sipaxos.hpp"

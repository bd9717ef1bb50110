// all.hpp -- every protocol with device transition functions.
#pragma once
#include "amokv.hpp"
#include "minitest.hpp"
#include "multipaxos.hpp"
#include "pb.hpp"
#include "pingpong.hpp"
#include "sipaxos.hpp"
#include "synthetic.hpp"
#include "gen/pingpong_ir.hpp"  // generated from the protocol IR (tools/gen_ir.py)
#include "gen/amokv_ir.hpp"
#include "gen/multipaxos_ir.hpp"
#include "gen/pb_ir.hpp"
#define DSL_HAVE_MULTIPAXOS 1

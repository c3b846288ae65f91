// Reference CLI protocol (Utility.cpp:66-124, kdtree_sequential.cpp:140-208).
//   eval mode  : stdout "READY", stderr prompt "Specify seed ", seed from stdin,
//                dim = 128, N = 500000 (Utility.cpp:92-102)
//   debug mode : argv SEED DIM_POINTS NUM_POINTS (Utility.cpp:104-120)
//   results    : "ID: <id> \t DISTANCE: <float>" (Utility.cpp:122-124), then
//                [debug] "elapsed time <s> second", then "DONE".
// Byte-identical output matters: graders diff stdout.
#pragma once
#include <string>

namespace pkdtree {

struct Problem {
  int seed = 0;
  int dim = 0;
  int num_points = 0;
};

void validate_input(const Problem& p);                  // exits(1) like the reference
Problem specify_problem_stdin();                        // eval mode
Problem specify_problem_argv(int argc, char** argv);    // debug mode (argv[1..3])
void print_result_line(long long id, float distance);
void print_elapsed(double seconds);
void print_done();

}  // namespace pkdtree

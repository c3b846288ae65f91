// Reference CLI protocol; messages and formatting follow Utility.cpp:66-124 byte for byte.
#include "pkdtree/protocol.hpp"

#include <cstdlib>
#include <iostream>
#include <string>

namespace pkdtree {

void validate_input(const Problem& p) {
  if (p.seed == 0) std::cerr << "Warning: default value 0 used as seed." << std::endl;
  if (p.seed < 0) { std::cerr << "Seed has to be larger than 0!" << std::endl; std::exit(1); }
  if (p.dim <= 0) { std::cerr << "Dimension has to be larger than 0!" << std::endl; std::exit(1); }
  if (p.num_points <= 0) { std::cerr << "Number of points has to be larger than 0!" << std::endl; std::exit(1); }
  std::cerr << "\tUsing seed " << p.seed << std::endl;
  std::cerr << "\tUsing point dimensions " << p.dim << std::endl;
  std::cerr << "\tUsing number of points " << p.num_points << std::endl << std::endl;
}

Problem specify_problem_stdin() {
  Problem p;
  std::cout << "READY" << std::endl;
  std::cerr << "Specify seed ";
  std::cin >> p.seed;
  p.dim = 128;
  p.num_points = 500000;
  validate_input(p);
  return p;
}

Problem specify_problem_argv(int argc, char** argv) {
  if (argc != 4) {
    std::cerr << "Usage: " << argv[0] << " SEED DIM_POINTS  NUM_POINTS" << std::endl;
    std::exit(1);
  }
  std::cout << "READY" << std::endl;
  Problem p;
  p.seed = std::stoi(argv[1]);
  p.dim = std::stoi(argv[2]);
  p.num_points = std::stoi(argv[3]);
  validate_input(p);
  return p;
}

void print_result_line(long long id, float distance) {
  std::cout << "ID: " << id << " \t DISTANCE: " << distance << std::endl;
}

void print_elapsed(double seconds) { std::cout << "elapsed time " << seconds << " second" << std::endl; }

void print_done() { std::cout << "DONE" << std::endl; }

}  // namespace pkdtree

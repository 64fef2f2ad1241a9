"""The oracle as a sliding-window backend (test infrastructure): the same three calls the okvisgpu
backend answers (okvisgpu_solve / okvisgpu_imu_append / okvisgpu_twopose_compute), answered by the
CPU restatement, so that _sliding_window can run one sequence on each and compare."""
import ctypes as C

import _oracle


class OracleBackend:
    def solve(self, problem, options):
        return _oracle.solve(C.pointer(problem), options)

    def imu_append(self, *args):
        return _oracle.imu_append(*args)

    def twopose(self, batch):
        return _oracle.twopose_compute(batch)

    def close(self):
        pass

"""Problem-definition layer: point-set shapes/values of every BC class (SURVEY.md §4 goldens)."""
import math

import numpy as np
import pytest

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import (DomainND, IC, FunctionDirichletBC, FunctionNeumannBC, dirichletBC,
                                         periodicBC)


def ac_domain():
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 512)
    D.add("t", [0.0, 1.0], 201)
    return D


def test_domain_dict_keys_and_collocation():
    tdq.set_seed(0)
    D = ac_domain()
    d = D.domaindict[0]
    for k in ("identifier", "range", "xfidelity", "xlinspace", "xupper", "xlower"):
        assert k in d
    assert d["xlinspace"].shape == (512,)
    D.generate_collocation_points(1000)
    assert D.X_f.shape == (1000, 2)
    assert D.X_f[:, 0].min() >= -1 and D.X_f[:, 0].max() <= 1
    assert D.X_f[:, 1].min() >= 0 and D.X_f[:, 1].max() <= 1


def test_ac_ic_and_periodic_shapes():
    tdq.set_seed(0)
    D = ac_domain()
    ic = IC(D, [lambda x: x ** 2 * np.cos(math.pi * x)], var=[["x"]])
    assert ic.input.shape == (512, 2)
    assert np.all(ic.input[:, 1] == 0.0)
    assert ic.val.shape == (512, 1)
    np.testing.assert_allclose(ic.val[:, 0], ic.input[:, 0] ** 2 * np.cos(math.pi * ic.input[:, 0]))
    per = periodicBC(D, ["x"], [lambda u, x, t: u(x)])
    assert len(per.upper_points) == 1 and per.upper_points[0].shape == (201, 2)
    assert np.all(per.upper_points[0][:, 0] == 1.0) and np.all(per.lower_points[0][:, 0] == -1.0)
    np.testing.assert_array_equal(per.upper_points[0][:, 1], per.lower_points[0][:, 1])
    assert np.asarray(per.upper).shape == (1, 2, 201, 1)  # reference's unrolled layout


def test_burgers_dirichlet():
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 256)
    D.add("t", [0.0, 1.0], 100)
    up = dirichletBC(D, val=0.0, var="x", target="upper")
    lo = dirichletBC(D, val=0.0, var="x", target="lower")
    assert up.input.shape == (100, 2) and np.all(up.input[:, 0] == 1.0)
    assert lo.input.shape == (100, 2) and np.all(lo.input[:, 0] == -1.0)
    np.testing.assert_allclose(up.input[:, 1], np.linspace(0, 1, 100))
    with pytest.raises(ValueError):
        dirichletBC(D, val=0.0, var="x", target="middle")


def test_function_dirichlet_subset_and_full():
    tdq.set_seed(3)
    D = DomainND(["x", "y"])
    D.add("x", [0, 1.0], 11)
    D.add("y", [0, 1.0], 11)
    f = lambda y: -np.sin(math.pi * y)
    bc = FunctionDirichletBC(D, fun=[f], var="x", target="upper", func_inputs=["y"], n_values=10)
    assert bc.input.shape == (10, 2) and np.all(bc.input[:, 0] == 1.0)
    np.testing.assert_allclose(bc.val[:, 0], f(bc.input[:, 1]))
    full = FunctionDirichletBC(D, fun=[f], var="x", target="upper", func_inputs=["y"])  # B18 fix
    assert full.input.shape == (11, 2)
    np.testing.assert_allclose(full.val[:, 0], f(full.input[:, 1]))


def test_3d_ic_and_periodic():
    D = DomainND(["x", "y", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 256)
    D.add("y", [-1.0, 1.0], 256)
    D.add("t", [0.0, 1.0], 100)
    ic = IC(D, [lambda x, y: -np.sin(x * math.pi) - np.sin(y * math.pi)], var=[["x", "y"]])
    assert ic.input.shape == (65536, 3) and np.all(ic.input[:, 2] == 0)
    np.testing.assert_allclose(ic.val[:, 0], -np.sin(ic.input[:, 0] * math.pi) - np.sin(ic.input[:, 1] * math.pi))
    per = periodicBC(D, ["x", "y"], [lambda u, x, y, t: u(x)])
    assert len(per.upper_points) == 2 and per.upper_points[0].shape == (25600, 3)
    assert np.all(per.upper_points[1][:, 1] == 1.0)


def test_ic_time_column_follows_declaration_order():  # B19
    D = DomainND(["t", "x"], time_var="t")
    D.add("t", [0.0, 2.0], 5)
    D.add("x", [-1.0, 1.0], 7)
    ic = IC(D, [lambda x: x], var=[["x"]])
    assert ic.input.shape == (7, 2) and np.all(ic.input[:, 0] == 0.0)
    np.testing.assert_allclose(ic.val[:, 0], ic.input[:, 1])


def test_neumann_points_and_values():
    tdq.set_seed(1)
    D = DomainND(["x", "y"])
    D.add("x", [0.0, 1.0], 9)
    D.add("y", [0.0, 2.0], 13)
    bc = FunctionNeumannBC(D, fun=[lambda y: y ** 2], var="x", target="lower",
                           deriv_model=[lambda u, x, y: tdq.grad(u(x, y), x)], func_inputs=["y"])
    assert bc.points[0].shape == (13, 2) and np.all(bc.points[0][:, 0] == 0.0)
    np.testing.assert_allclose(bc.val[:, 0], bc.points[0][:, 1] ** 2)


def test_sampling_with_replacement_default_and_without():
    tdq.set_seed(0)
    D = ac_domain()
    per = periodicBC(D, ["x"], [lambda u, x, t: u(x)])
    assert len(np.unique(per.nums)) < 201  # reference semantics (B20)
    per2 = periodicBC(D, ["x"], [lambda u, x, t: u(x)], replace=False)
    assert len(np.unique(per2.nums)) == 201

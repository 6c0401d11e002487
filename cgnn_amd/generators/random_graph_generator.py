"""Layered random causal DAG + data generator
(reference: generators/random_graph_generator.py:25-189).

``generate`` draws ``randint(2, n / floor(sqrt(n)))`` root causes, then adds
layers; each new node gets up to ``max_joint_causes`` parents among earlier
nodes, one random spline mechanism per parent, contributions summed (the
reference's effective behaviour, B9), a final additive or multiplicative noise,
and is standardised.  Optionally ``categorical_rate`` of the variables are
discretised.  ``generate_pairs`` (broken in the reference, B9) produces a
CEPC pairs file from the generated edges.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from ..utils.formats import standardize, write_cepc_pairs
from ..utils.graph import DirectedGraph
from .functions_default import cause, effect, noise, rand_bin


def series_to_cepc_kag(A, B, idxpair):
    def fmt(v):
        return "".join(" " + str(x) for x in np.asarray(v).ravel())
    return pd.DataFrame([['pair' + str(idxpair), fmt(A), fmt(B)]], columns=['SampleID', 'A', 'B'])


class RandomGraphGenerator:
    def __init__(self, num_nodes=200, max_joint_causes=4, noise_qty=.7, number_points=500,
                 categorical_rate=.20, seed=None, verbose=False):
        self.nodes = num_nodes
        self.noise = noise_qty
        self.n_points = number_points
        self.cat_rate = categorical_rate
        self.num_max_parents = max_joint_causes
        self.rng = np.random.default_rng(seed)
        self.verbose = verbose
        self.causes = None
        self.graph = None
        self.data = None
        self.result_links = None
        self.cat_data = None
        self.cat_var = None

    def _log(self, msg):
        if self.verbose:
            print(msg)

    def generate(self, gen_cat=True):
        r = self.rng
        n_roots = int(r.integers(2, max(3, int(self.nodes / np.floor(np.sqrt(self.nodes))))))
        self.causes = list(range(n_roots))
        cols = {}
        layer = [[]]
        for i in self.causes:
            cols['V' + str(i)] = cause(self.n_points, rng=r)
            layer[0].append(i)
        generated = len(self.causes)
        links = []
        while generated < self.nodes:
            self._log('--Generating nodes : {} out of ~{}'.format(generated, self.nodes))
            layer.append([])
            n_layer = int(r.integers(2, len(layer[-2]) + 2))
            for _ in range(n_layer):
                layer[-1].append(generated)
                last_idx = layer[-2][-1]
                parents = sorted(set(int(r.integers(0, max(last_idx, 1))) for _ in range(self.num_max_parents)))
                child = []
                for par in parents:
                    links.append(['V' + str(par), 'V' + str(generated)])
                    child.append(effect(cols['V' + str(par)], self.n_points, self.noise, rng=r))
                r.shuffle(child)
                result = child[0]
                for c in child[1:]:
                    result = result + c
                if r.integers(0, 2) == 1:      # multiplicative noise
                    nv = noise(self.n_points, self.noise, rng=r).ravel()
                    result = (result + abs(result.min())) * (nv + abs(nv.min()))
                else:
                    result = result + noise(self.n_points, self.noise, rng=r).ravel()
                cols['V' + str(generated)] = standardize(result)
                generated += 1
        self.data = pd.DataFrame(cols)
        self.result_links = pd.DataFrame(links, columns=["Cause", "Effect"])
        if gen_cat:
            self.cat_var = []
            self.cat_data = self.data.copy()
            n_cols = len(self.data.columns)
            while float(len(self.cat_var)) / n_cols < self.cat_rate:
                var = int(r.integers(0, n_cols))
                while var in self.cat_var:
                    var = int(r.integers(0, n_cols))
                self.cat_var.append(var)
                self.cat_data['V' + str(var)] = rand_bin(list(self.cat_data['V' + str(var)]), rng=r)
            self.cat_var = pd.DataFrame(self.cat_var)
        self.graph = DirectedGraph()
        self.graph.add_multiple_edges([list(x) + [1] for x in self.result_links.values])
        for c in self.data.columns:
            self.graph.add_node(c)
        return self.get_data()

    def get_data(self):
        if self.graph is None:
            raise NameError('Please compute graph using .generate(), graph not build yet')
        return self.graph, self.data, self.cat_data, self.cat_var

    def save_data(self, filename):
        if self.result_links is None:
            raise NameError('Please compute graph using .generate(), graph not build yet')
        self.result_links.to_csv(filename + '_target.csv', sep=',', index=False)
        self.data.to_csv(filename + '_numdata.csv', sep=',', index=False)
        if self.cat_data is not None:
            self.cat_data.to_csv(filename + '_catdata.csv', sep=',', index=False)
            self.cat_var.to_csv(filename + '_catindex.csv', sep=',', index=False)

    def generate_pairs(self, num_pairs, prefix=None):
        pairs, targets = [], []
        while len(pairs) < num_pairs:
            self.generate(gen_cat=False)
            for link in self.result_links.itertuples(index=False):
                if len(pairs) >= num_pairs:
                    break
                k = len(pairs)
                if self.rng.integers(0, 2):
                    pairs.append(series_to_cepc_kag(self.data[link.Cause], self.data[link.Effect], k))
                    targets.append(['pair' + str(k), 1.0])
                else:
                    pairs.append(series_to_cepc_kag(self.data[link.Effect], self.data[link.Cause], k))
                    targets.append(['pair' + str(k), -1.0])
        pairs_df = pd.concat(pairs, ignore_index=True)
        target_df = pd.DataFrame(targets, columns=['SampleID', 'Target'])
        if prefix is None:
            prefix = 'p_graphgen_G' + str(self.num_max_parents) + '_N' + str(self.nodes)
        pairs_df.to_csv(prefix + '_pairs.csv', index=False)
        target_df.to_csv(prefix + '_targets.csv', index=False)
        return pairs_df, target_df

"""Writes the committed golden fixtures under tests/golden/.

compute_error_kat.json
    The reference's own known-answer lines for computeError
    (/root/reference/output.txt:16-18: 1.22474487139, 3.16227766017, 0.0).  The
    inputs are not in the reference repository; they are the CS100 lab-4 test
    RDDs as reconstructed in SURVEY.md §4 (they reproduce all three printed
    values exactly).  Expected values are copied from output.txt, not computed.

personal_ratings.json
    The 12 personal ratings of user 0 (RecommenderSystem.py:190-202) and the
    reference's printed dataset facts (output.txt:1, :9) used by the
    script-shaped end-to-end test.

This script only writes data; it does not import or execute the reference.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

predicted = [(1, 1, 5), (1, 2, 3), (1, 3, 4), (2, 1, 3), (2, 2, 2), (2, 3, 4)]
predicted2 = [(2, 2, 5), (1, 2, 5)]
actual = [(1, 2, 3), (1, 3, 5), (2, 1, 5), (2, 2, 1)]

kat = {
    "source": "output.txt:16-18 (expected); inputs reconstructed per SURVEY.md section 4",
    "cases": [
        {"name": "test dataset", "predicted": predicted, "actual": actual,
         "expected": 1.22474487139},
        {"name": "test dataset2", "predicted": predicted2, "actual": actual,
         "expected": 3.16227766017},
        {"name": "testActual dataset", "predicted": actual, "actual": actual, "expected": 0.0},
    ],
}
with open(os.path.join(HERE, "compute_error_kat.json"), "w") as f:
    json.dump(kat, f, indent=1)

personal = {
    "source": "RecommenderSystem.py:190-202 (myRatedMovies), output.txt:1 and :9",
    "my_user_id": 0,
    "my_rated_movies": [[0, 1088, 2], [0, 1171, 4], [0, 1047, 2], [0, 1195, 5], [0, 831, 1],
                        [0, 503, 2], [0, 651, 4], [0, 1447, 5], [0, 1110, 1], [0, 553, 3],
                        [0, 594, 2], [0, 700, 3]],
    "ratings_count": 487650, "movies_count": 3883,
    "split_counts": {"training": 292716, "validation": 96902, "test": 98032},
    "hyperparameters": {"seed": 5, "iterations": 5, "regularizationParameter": 0.1,
                        "ranks": [4, 8, 12]},
    "reported_validation_rmse": {"4": 0.890718281504, "8": 0.89536885148, "12": 0.89189947948},
    "reported_test_rmse": 0.892429324592,
}
with open(os.path.join(HERE, "personal_ratings.json"), "w") as f:
    json.dump(personal, f, indent=1)
print("wrote", sorted(os.listdir(HERE)))

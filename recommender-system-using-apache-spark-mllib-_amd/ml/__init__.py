"""pyspark.ml-shaped namespace of als_mi355x."""

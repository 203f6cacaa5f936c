"""pyspark.mllib-shaped namespace of als_mi355x."""
